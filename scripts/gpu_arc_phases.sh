#!/bin/bash
# arc_kernel phase cut-offs (ECC_ARC_DBG: 3 = setup, 2 = +staging, 1 = +fill/prefix, 0 = full) under the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for d in ${ARC_DBG_MODES:-0 1 2 3}; do
  ECC_ARC_DBG=$d timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --no-tracker --no-ingest > gpurun_out/arc_dbg$d.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/arc_dbg$d.json'));print('dbg=$d', d['stages_ms_per_step']['arc_kernel'])"
done
