#!/bin/bash
# Downsample grid-stride variants: parity on each, then the headline-step A/B.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO" && mkdir -p gpurun_out
PKG="$REPO/event-camera-clustering-and-optical-flow-estimation_amd"
for v in lib lib_d768 lib_d512; do
  ECC_LIB="$PKG/$v/libecc.so" timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "downsample or hash" > gpurun_out/ds_pytest.log 2>&1; rc=$?
  echo "$v $(tail -1 gpurun_out/ds_pytest.log)"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_variants_ab.sh lib_d768 lib_d512
