#!/bin/bash
# round-3 first GPU session: the new sharded-step GPU tests, then one default bench run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_dist.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err; rc=$?
echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_r03a.json; tail -5 gpurun_out/bench_r03a.err
