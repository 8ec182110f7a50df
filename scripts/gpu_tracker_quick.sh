#!/bin/bash
# Tracker parity subset + the bench's tracker timing.  Usage: gpu_tracker_quick.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tracker" > gpurun_out/pytest_tracker.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_tracker.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_tracker.json 2> gpurun_out/bench_tracker.err; rc=$?
echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/bench_tracker.json'));print('tracker_us_per_slice',d['tracker_us_per_slice'],'value',d['value'])"
