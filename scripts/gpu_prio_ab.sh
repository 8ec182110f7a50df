#!/bin/bash
# A/B of the k-means stream priority in the single-GPU step (headline only, no side measurements).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for p in 1 0 -1 1 0; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-tracker --no-ingest --no-eps --no-c3 --kmeans-priority $p > gpurun_out/prio_$p.json 2> gpurun_out/prio_$p.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/prio_$p.json'));print('prio $p', d['value'], d['ms_per_step'])"
done
