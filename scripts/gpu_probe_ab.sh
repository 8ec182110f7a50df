#!/bin/bash
# A/B of one probe under rocprofv3 --kernel-trace --stats: the default libecc (a) against lib_exp (b).
# Usage: gpu_probe_ab.sh <tag> <probe.py> [args...]
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
P="$REPO/scripts/$1"; shift
OUT="$REPO/gpurun_out/ab_$TAG"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
PKG="$REPO/event-camera-clustering-and-optical-flow-estimation_amd"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$OUT/a" -o a --output-format csv -- python3 "$P" "$@" > "$OUT/a.log" 2>&1 || exit $?
ECC_LIB="$PKG/lib_exp/libecc.so" timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$OUT/b" -o b --output-format csv -- python3 "$P" "$@" > "$OUT/b.log" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, sys, glob
out = sys.argv[1]
for tag in ("a", "b"):
    for r in csv.DictReader(open(glob.glob(f"{out}/{tag}/*kernel_stats.csv")[0])):
        print(tag, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
