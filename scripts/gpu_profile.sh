#!/bin/bash
# rocprofv3 session: kernel trace + stats of the bench, then separate PMC passes for HBM
# traffic (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  Counter passes use
# --kernel-trace only (never sys/runtime traces with --pmc).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"; shift
ARGS="--steps 3 --warmup 1 --no-cpu --no-tracker --serial $*"
OUT="$REPO/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
fault() { case "$1" in 0) return 0;; *) echo "rc=$1, stopping"; exit "$1";; esac; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 "$REPO/bench.py" $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace.err"; rc=$?; echo "trace rc=$rc"; fault $rc
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 "$REPO/bench.py" $ARGS > /dev/null 2> "$OUT/fetch.err"; rc=$?; echo "fetch rc=$rc"; fault $rc
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 "$REPO/bench.py" $ARGS > /dev/null 2> "$OUT/write.err"; rc=$?; echo "write rc=$rc"; fault $rc
find "$OUT" -name "*.csv" | head -20
