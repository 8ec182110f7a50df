#!/bin/bash
# round 3 (i): the whole -m gpu suite + bench (gpu_session.sh), then the list-chain and f32
# k-means counter passes.  Stops at the first GPU fault, abort or timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash scripts/gpu_session.sh ${TAG:-r03i}; rc=$?
case $rc in 0|1) ;; *) echo "session rc=$rc: stopping"; exit $rc;; esac
bash scripts/gpu_pmc_lists.sh > gpurun_out/pmc_lists.txt 2>&1; r=$?; echo "lists rc=$r"; [ $r -eq 0 ] || exit $r
bash scripts/gpu_pmc_kmf32.sh > gpurun_out/pmc_kmf32.txt 2>&1; r=$?; echo "kmf32 rc=$r"; [ $r -eq 0 ] || exit $r
exit $rc
