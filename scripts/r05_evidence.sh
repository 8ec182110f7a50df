#!/bin/bash
# Round evidence at HEAD in one GPU call: the -m gpu suite, scripts/gpu_evidence.sh (rocprof trace +
# stats, FETCH/WRITE traffic, SQ occupancy, calibration, the default bench line), then SQ/traffic
# passes over the DBSCAN kernels (eps_probe.py dbscan / lists).  Every step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="$1"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest.log
bash scripts/gpu_evidence.sh "$TAG" || exit 1
bash scripts/gpu_pmc.sh "db_$TAG" eps_probe.py dbscan || exit 1
bash scripts/gpu_pmc.sh "lists_$TAG" eps_probe.py lists || exit 1
