#!/bin/bash
# GPU test session: the full -m gpu suite (one process), then smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -m gpu -q -rf "$@" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/smoke.log
