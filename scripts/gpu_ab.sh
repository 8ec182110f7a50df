#!/bin/bash
# The -m gpu suite on the default library (skipped with NO_TESTS=1), then a two-round bench A/B of
# lib against the library variants lib_<v> built by scripts/mkvar.sh / mkflag.sh:
#   gpu_ab.sh <tag> <variant>... [-- extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="$1"; shift
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; [ "$1" = "--" ] && shift
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -n 1 gpurun_out/${TAG}_pytest.log
fi
bash scripts/ab_libs.sh "$TAG" --steps 20 --warmup 5 --no-cpu --no-ingest --no-c3 "$@" -- "${V[@]}"
