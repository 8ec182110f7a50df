#!/bin/bash
# Fused detect + NMS: the NMS / fast_detect parity subset, then the headline step in both schedules.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "nms or fast_detect or corner or smoke" > gpurun_out/fused_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/fused_pytest.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 20 --warmup 5 --no-cpu --no-tracker --no-ingest --no-eps --no-c3"
for mode in --serial ""; do
  timeout -k 10 300 python3 bench.py $ARGS $mode > gpurun_out/fused_b.json 2> gpurun_out/fused_b.err || { echo "bench rc=$?"; tail -5 gpurun_out/fused_b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/fused_b.json').read().strip().splitlines()[-1]);print('${mode:-two-stream}', d['ms_per_step'], d['stages_ms_per_step'])"
done
