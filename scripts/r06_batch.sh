#!/bin/bash
# One GPU call for several variant experiments (each step under its own limit; stops at the first
# failure): parity of each variant library on the tests it touches, then its bench / probe numbers.
#   r06_batch.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
T="$1"; L=$PWD/event-camera-clustering-and-optical-flow-estimation_amd
fault() { case "$1" in 0) return 0;; *) echo "rc=$1 at $2, stopping"; exit "$1";; esac; }
pt() {  # pt <lib> <log> <pytest args...>
  local lib="$1" log="$2"; shift 2
  ECC_LIB=$L/$lib/libecc.so timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread "$@" > gpurun_out/${T}_$log.log 2>&1
  local rc=$?; tail -1 gpurun_out/${T}_$log.log; [ $rc = 0 ] || tail -25 gpurun_out/${T}_$log.log; return $rc
}
pt lib base tests/test_gpu_parity.py tests/test_gpu_c4_full.py tests/test_gpu_clouds.py -k "count_images or dbscan or c4 or fast_detect or dense"; fault $? base
pt lib_t256 t256 tests/test_gpu_state.py tests/test_gpu_c4_full.py tests/test_gpu_parity.py -k "track or c4 or state"; fault $? t256
pt lib_dn1k dn1k tests/test_gpu_c4_full.py tests/test_gpu_parity.py -k "c4 or fast_detect or dense"; fault $? dn1k
pt lib_un2 un2 tests/test_gpu_parity.py tests/test_gpu_clouds.py -k "dbscan"; fault $? un2
for v in lib lib_t256; do ECC_LIB=$L/$v/libecc.so timeout -k 10 120 python scripts/tracker_probe.py > gpurun_out/${T}_trk_$v.txt 2>&1; fault $? trk_$v; tail -1 gpurun_out/${T}_trk_$v.txt | cut -c1-40; done
timeout -k 10 200 python scripts/step_probe.py 20 > gpurun_out/${T}_step.txt 2>&1; fault $? step; tail -6 gpurun_out/${T}_step.txt
NO_TESTS=1 bash scripts/gpu_ab.sh $T lib_dn1k lib_un2 -- --no-tracker; fault $? ab
