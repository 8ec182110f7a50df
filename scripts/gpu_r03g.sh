#!/bin/bash
# round 3 (g): eps/dbscan/downsample/k-means GPU tests, then the list-chain and f32 k-means
# profiles.  Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
LOG_NAME=pytest_r03g TMO=400 bash scripts/gpu_tests.sh tests/test_gpu_parity.py tests/test_gpu_clouds.py \
    -k "eps or dbscan or optics or downsample or hash or kmeans" || exit $?
bash scripts/gpu_pmc_lists.sh > gpurun_out/pmc_lists.txt 2>&1; rc=$?; echo "lists rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_kmf32.sh > gpurun_out/pmc_kmf32.txt 2>&1; rc=$?; echo "kmf32 rc=$rc"; exit $rc
