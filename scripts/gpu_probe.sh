#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for d in 0 1 2 4 8; do echo "== DBG $d"; ECC_CORNER_DBG=$d timeout -k 10 120 python scripts/corner_probe.py | grep total | cut -c1-60 || exit $?; done
