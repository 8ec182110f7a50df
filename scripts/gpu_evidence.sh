#!/bin/bash
# Round evidence for the bench workload in one GPU call, every step under its own time limit:
#   1. rocprofv3 kernel trace + stats of `bench.py --serial` (per-kernel durations);
#   2. FETCH_SIZE and WRITE_SIZE passes (HBM traffic, scripts/traffic.py);
#   3. two SQ counter passes (occupancy, wait and issue fractions: scripts/pmc_summary.py);
#   4. the FETCH_SIZE / WRITE_SIZE calibration of scripts/calib/fetch_calib (known byte counts);
#   5. the default bench line.
# PMC passes use --kernel-trace only (never sys/runtime traces with --pmc).
# Usage: gpu_evidence.sh <tag> [extra bench args]      (SKIP_BENCH=1 skips step 5)
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r04}"; shift
ARGS="--steps 3 --warmup 1 --no-cpu --no-tracker --no-eps --no-c3 --no-ingest --serial $*"
OUT="$REPO/gpurun_out/ev_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
fault() { case "$1" in 0) return 0;; *) echo "rc=$1 at $2, stopping"; exit "$1";; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 "$REPO/bench.py" $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace.err"; fault $? trace
python3 -c 'import hashlib, json, sys; print(json.dumps({"libecc_sha256": hashlib.sha256(open(sys.argv[1], "rb").read()).hexdigest(), "command": sys.argv[2]}))' \
  "${ECC_LIB:-$REPO/event-camera-clustering-and-optical-flow-estimation_amd/lib/libecc.so}" "bench.py $ARGS" > "$OUT/kernel_stats.meta.json"
echo "trace done"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 "$REPO/bench.py" $ARGS > /dev/null 2> "$OUT/fetch.err"; fault $? fetch
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 "$REPO/bench.py" $ARGS > /dev/null 2> "$OUT/write.err"; fault $? write
echo "traffic done"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P1 -d "$OUT/sq/p1" -o p --output-format csv -- python3 "$REPO/bench.py" $ARGS > /dev/null 2> "$OUT/sq1.err"; fault $? sq1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P2 -d "$OUT/sq/p2" -o p --output-format csv -- python3 "$REPO/bench.py" $ARGS > /dev/null 2> "$OUT/sq2.err"; fault $? sq2
echo "sq done"
if [ -x "$REPO/scripts/calib/bin/fetch_calib" ]; then
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/calib_fetch" -o c --output-format csv -- "$REPO/scripts/calib/bin/fetch_calib" > "$OUT/calib_bytes.txt" 2> "$OUT/calib_fetch.err"; fault $? calib_fetch
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/calib_write" -o c --output-format csv -- "$REPO/scripts/calib/bin/fetch_calib" > /dev/null 2> "$OUT/calib_write.err"; fault $? calib_write
  echo "calib done"
fi
cd "$REPO"
python3 scripts/traffic.py "$OUT" "$OUT/traffic.json" > "$OUT/traffic.txt" || exit 1
python3 scripts/pmc_summary.py "$OUT/sq" "$OUT/occupancy.json" > "$OUT/occupancy.txt" || exit 1
[ -x scripts/calib/bin/fetch_calib ] && { python3 scripts/calib_report.py "$OUT" > "$OUT/calib.txt" || exit 1; }
cat "$OUT/traffic.txt" "$OUT/occupancy.txt" "$OUT/calib.txt" 2>/dev/null | head -80
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"; fault $? bench
head -c 600 "$OUT/bench.json"
