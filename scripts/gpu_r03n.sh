#!/bin/bash
# Round-3 close: pair_build 512-lane variant (lib_v1) parity + step A/B, then the round evidence.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO" && mkdir -p gpurun_out
PKG="$REPO/event-camera-clustering-and-optical-flow-estimation_amd"
ECC_LIB="$PKG/lib_v1/libecc.so" timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "fast_detect or corner" > gpurun_out/v1_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/v1_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_variants_ab.sh lib_v1 || exit $?
bash scripts/gpu_round.sh r03n
