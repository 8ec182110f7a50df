#!/bin/bash
# round-3 session: new cloud/state/k-means tests, then a bench run (CPU leg off)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
LOG_NAME=r03c TMO=900 bash scripts/gpu_tests.sh tests/test_gpu_state.py tests/test_gpu_clouds.py tests/test_host_programs.py tests/test_gpu_parity.py -k "dbscan or optics or radius or eps or kdtree or cloud or program or tracker or kmeans" || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_r03c.json 2> gpurun_out/bench_r03c.err; rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_r03c.json; tail -3 gpurun_out/bench_r03c.err
