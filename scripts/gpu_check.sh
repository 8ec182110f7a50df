#!/bin/bash
# One GPU session: parity tests, smoke, bench.  Stops at the first fault/abort/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fault() { # $1 = rc ; faults/timeouts end the session
  case "$1" in 0|1|2|5) return 0;; *) echo "fault rc=$1, stopping"; exit "$1";; esac
}
timeout -k 10 120 clinfo > gpurun_out/clinfo.txt 2>&1; echo "clinfo rc=$?"
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; stop_if_fault $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; stop_if_fault $rc
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
