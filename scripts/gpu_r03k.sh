#!/bin/bash
# round 3 (k): rocprofv3 kernel stats + HBM traffic passes of the bench (gpu_profile.sh), then the
# corner stage's SQ counters.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash scripts/gpu_profile.sh r03k > gpurun_out/prof_r03k.txt 2>&1; rc=$?; echo "profile rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_corner.sh > gpurun_out/pmc_corner_r03k.txt 2>&1; rc=$?; echo "corner pmc rc=$rc"; exit $rc
