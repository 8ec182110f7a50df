#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "fast or arc or handoff or corner" > gpurun_out/pytest_probe.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_probe.log; [ $rc -le 1 ] || exit $rc
for d in 0 2 4; do echo "== DBG $d"; ECC_CORNER_DBG=$d timeout -k 10 120 python scripts/corner_probe.py || exit $?; done
