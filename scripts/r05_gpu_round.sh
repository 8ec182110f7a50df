#!/bin/bash
# One GPU call: the -m gpu suite, then (only if green) the probes and two bench runs.
# Every GPU step has its own time limit; a step that fails stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="${1:-r05}"
fault() { case "$1" in 0) return 0;; *) echo "rc=$1 at $2, stopping"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; fault $? pytest
tail -n 2 gpurun_out/${TAG}_pytest.log
L=$PWD/event-camera-clustering-and-optical-flow-estimation_amd/lib_prof/libecc.so
ECC_LIB=$L timeout -k 10 120 python scripts/tracker_probe.py > gpurun_out/${TAG}_trk.txt 2>&1; fault $? trk
tail -n 2 gpurun_out/${TAG}_trk.txt
ECC_LIB=$L timeout -k 10 120 python scripts/eps_probe.py dbscan > gpurun_out/${TAG}_db.txt 2>&1; fault $? db
tail -n 1 gpurun_out/${TAG}_db.txt
ECC_LIB=$L timeout -k 10 120 python scripts/arc_probe.py > gpurun_out/${TAG}_arc.txt 2>&1; fault $? arc
tail -n 1 gpurun_out/${TAG}_arc.txt
bash scripts/ab_libs.sh ${TAG} --steps 20 --warmup 5 --no-cpu --no-ingest --no-c3 -- ; fault $? bench
