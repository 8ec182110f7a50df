#!/bin/bash
# Quick loop: a subset of the parity suite (-k expr in $1) + the bench without CPU baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "${1:-kmeans}" > gpurun_out/pytest_quick.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-tracker > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err; rc=$?; echo "bench rc=$rc"
python -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));print(d['value'],d['ms_per_step']);print(json.dumps(d['stages_ms_per_step']))"
