#!/bin/bash
# Quick loop: a parity subset (-k expr in $1), then the bench twice without CPU baseline/tracker/
# ingest: --serial (one stream: isolated per-kernel times) and the default two-stream step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "${1:-fast_detect or arc or nms or corner or sae or smoke}" > gpurun_out/pq.log 2>&1; rc=$?
tail -15 gpurun_out/pq.log; [ $rc -eq 0 ] || exit $rc
for mode in --serial ""; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-tracker --no-ingest --no-eps $mode > gpurun_out/bq.json 2> gpurun_out/bq.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/bq.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bq.json'));print('${mode:-two-stream}', d['value'],d['ms_per_step']);print(json.dumps(d['stages_ms_per_step'])) if '$mode' else None"
done
