#!/bin/bash
# GPU test session: pytest over the given arguments (default: the whole -m gpu suite), one process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
LOG=gpurun_out/${LOG_NAME:-pytest_gpu}.log
timeout -k 10 ${TMO:-900} python -u -m pytest -m gpu -x -v -rf --timeout 300 --timeout-method thread "${@:-tests}" > "$LOG" 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" "$LOG" | tail -40
exit $rc
