#!/bin/bash
# GPU session: the whole -m gpu suite, then (only when pytest ran to an ordinary end: all passed or
# test failures, never after a crash or timeout) one bench run with BENCH_ARGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="${1:-sess}"
LOG_NAME="pytest_$TAG" TMO="${TMO:-900}" bash scripts/gpu_tests.sh ${TESTS:-tests}; rc=$?
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 600 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:---no-cpu} > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err"; brc=$?
echo "bench rc=$brc"; tail -c 300 "gpurun_out/bench_$TAG.json"; tail -3 "gpurun_out/bench_$TAG.err"
exit $(( rc > brc ? rc : brc ))
