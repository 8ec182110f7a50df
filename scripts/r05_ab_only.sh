#!/bin/bash
# Two-round bench A/B (corner focus) of lib against the variants in $@, no tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="$1"; shift
bash scripts/ab_libs.sh ${TAG} --steps 20 --warmup 5 --no-cpu --no-ingest --no-c3 --no-eps --no-tracker -- "$@"
