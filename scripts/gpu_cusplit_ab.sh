#!/bin/bash
# A/B of the single-GPU step with the k-means chain on N dedicated CUs (0 = shared).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for c in 0 16 24 32 48 64 0 32; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-tracker --no-ingest --no-eps --no-c3 --kmeans-cus $c > gpurun_out/cus_$c.json 2> gpurun_out/cus_$c.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/cus_$c.json'));print('cus $c', d['value'], d['ms_per_step'], d['parity'] if 'parity' in d else '')"
done
