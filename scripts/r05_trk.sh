#!/bin/bash
# tracker phase split (profiling builds) for each library dir in $@
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG=$1; shift
for v in "$@"; do echo "== $v"; ECC_LIB=$PWD/event-camera-clustering-and-optical-flow-estimation_amd/$v/libecc.so timeout -k 10 120 python scripts/tracker_probe.py > gpurun_out/${TAG}_trk_$v.txt 2>&1 || { tail -5 gpurun_out/${TAG}_trk_$v.txt; exit 1; }; cat gpurun_out/${TAG}_trk_$v.txt; done
