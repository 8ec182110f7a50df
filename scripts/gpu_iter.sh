#!/bin/bash
# Iteration GPU session: selected -m gpu tests (-k EXPR, default all), optional dist rehearsal
# (DIST=1), then one default bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
K="${1:-}"
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_iter.log 2>&1; rc=$?
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?
fi
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_iter.log
case $rc in 0|1|5) ;; *) exit $rc;; esac
if [ "${DIST:-0}" = 1 ]; then bash scripts/gpu_dist_rehearsal.sh || exit $?; fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err; rc=$?
  echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_iter.json; tail -5 gpurun_out/bench_iter.err
fi
