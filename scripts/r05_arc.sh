#!/bin/bash
# The -m gpu suite, the arc phase probe (profiling lib), then a bench A/B of lib against $@.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="$1"; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest.log
L=$PWD/event-camera-clustering-and-optical-flow-estimation_amd/lib_prof/libecc.so
ECC_LIB=$L timeout -k 10 120 python scripts/arc_probe.py > gpurun_out/${TAG}_arc.txt 2>&1 || { echo "arc probe rc=$?"; tail -5 gpurun_out/${TAG}_arc.txt; exit 1; }
tail -n 1 gpurun_out/${TAG}_arc.txt
bash scripts/ab_libs.sh ${TAG} --steps 20 --warmup 5 --no-cpu --no-ingest --no-c3 --no-eps --no-tracker -- "$@"
