#!/bin/bash
# the wide-range corner cases on each library variant in $@, then the corner tests and a bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG=$1; shift
for v in lib "$@"; do echo "== $v"; ECC_LIB=$PWD/event-camera-clustering-and-optical-flow-estimation_amd/$v/libecc.so timeout -k 10 120 python scripts/dbg_wide.py > gpurun_out/${TAG}_dbg_$v.txt 2>&1 || exit 1; grep -c 'diff 0 ' gpurun_out/${TAG}_dbg_$v.txt; done
bash scripts/r05_corner.sh "$TAG" "$@"
