#!/bin/bash
# tracker GPU tests (default lib), then the tracker phase split of the profiling lib and the bench tracker key
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tracker or c4 or track" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest.log
bash scripts/r05_trk.sh "$TAG" "$@"
