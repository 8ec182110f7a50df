#!/bin/bash
# Round 3: the k-means candidate table — k-means parity tests, then the C3 probe's kernel stats and
# SQ counters (gpu_pmc_kmf32.sh).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k kmeans > gpurun_out/r03l_pytest.log 2>&1 || { tail -30 gpurun_out/r03l_pytest.log; exit 1; }
tail -3 gpurun_out/r03l_pytest.log
bash scripts/gpu_pmc_kmf32.sh > gpurun_out/r03l_pmc.txt 2>&1 || { tail -20 gpurun_out/r03l_pmc.txt; exit 1; }
cat gpurun_out/r03l_pmc.txt
