#!/bin/bash
# k-means GPU tests with each library variant in $@ (ECC_LIB), then a bench A/B of lib against them
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG=$1; shift
for v in "$@"; do
  ECC_LIB=$PWD/event-camera-clustering-and-optical-flow-estimation_amd/$v/libecc.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "kmeans or c4 or smoke or graph" > gpurun_out/${TAG}_pytest_$v.log 2>&1 || { echo "$v pytest rc=$?"; tail -20 gpurun_out/${TAG}_pytest_$v.log; exit 1; }
  echo "$v: $(tail -n 1 gpurun_out/${TAG}_pytest_$v.log)"
done
bash scripts/ab_libs.sh ${TAG} --steps 20 --warmup 5 --no-cpu --no-ingest --no-c3 --no-eps --no-tracker -- "$@"
