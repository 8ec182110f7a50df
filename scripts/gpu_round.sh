#!/bin/bash
# One GPU call for a round's evidence at the working tree's library, every GPU step under its own
# time limit, stopping at the first failure:
#   gpu_round.sh <tag> [tests|evidence|final|all]   (default: all)
#   tests:    the -m gpu suite (one pytest process)
#   evidence: scripts/gpu_evidence.sh (rocprof trace + stats + meta, FETCH/WRITE traffic, SQ
#             occupancy, calibration, a 20-step bench line), then SQ/traffic passes over the DBSCAN
#             row-run kernel and the list chain (scripts/eps_probe.py)
#   final:    __graft_entry__.smoke() on cuda:0 and the default bench line (what the driver runs)
# Copy the results into profiles/ with scripts/collect_evidence.sh <tag>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="$1"; WHAT="${2:-all}"
fault() { case "$1" in 0) return 0;; *) echo "rc=$1 at $2, stopping"; exit "$1";; esac; }
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1; fault $? pytest
  tail -n 1 gpurun_out/${TAG}_pytest.log
fi
if [ "$WHAT" = evidence ] || [ "$WHAT" = all ]; then
  bash scripts/gpu_evidence.sh "$TAG"; fault $? evidence
  bash scripts/gpu_pmc.sh "db_$TAG" eps_probe.py dbscan; fault $? pmc_db
  bash scripts/gpu_pmc.sh "lists_$TAG" eps_probe.py lists; fault $? pmc_lists
fi
if [ "$WHAT" = final ] || [ "$WHAT" = all ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/${TAG}_smoke.log 2>&1; fault $? smoke
  tail -n 1 gpurun_out/${TAG}_smoke.log
  timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; fault $? bench
  head -c 400 gpurun_out/${TAG}_bench.json
fi
