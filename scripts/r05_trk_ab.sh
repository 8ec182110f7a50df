#!/bin/bash
# tracker GPU tests on each library dir in $@ (ECC_LIB), then the tracker probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG=$1; shift
for v in "$@"; do
  ECC_LIB=$PWD/event-camera-clustering-and-optical-flow-estimation_amd/$v/libecc.so timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "tracker or c4 or track" > gpurun_out/${TAG}_pytest_$v.log 2>&1; echo "$v pytest rc=$?"; tail -n 3 gpurun_out/${TAG}_pytest_$v.log
  ECC_LIB=$PWD/event-camera-clustering-and-optical-flow-estimation_amd/$v/libecc.so timeout -k 10 120 python scripts/tracker_probe.py 300 > gpurun_out/${TAG}_trk_$v.txt 2>&1 || exit 1; head -2 gpurun_out/${TAG}_trk_$v.txt
done
