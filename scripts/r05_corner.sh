#!/bin/bash
# Corner-side GPU tests (default lib), then a two-round bench A/B of lib against the variants in $@.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="$1"; shift
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c4_full.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "fast_detect or arc or nms or c4 or corner or graph" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest.log
bash scripts/ab_libs.sh ${TAG} --steps 20 --warmup 5 --no-cpu --no-ingest --no-c3 --no-eps --no-tracker -- "$@"
