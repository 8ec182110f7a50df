#!/bin/bash
# Phase cut-offs of one kernel under the bench: ECC_ARC_DBG=<mode> for each mode in $2, reporting
# the per-step time of kernel $1 (the cut kernels' outputs are invalid; timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for d in $2; do
  ECC_ARC_DBG=$d timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --no-tracker --no-ingest > gpurun_out/dbg$d.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/dbg$d.json'));print('dbg=$d', d['stages_ms_per_step']['$1'])"
done
