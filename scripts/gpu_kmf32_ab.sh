#!/bin/bash
# A/B of the C3 f32 vector engine: the default libecc against lib_exp (built with
# `make KM_ACC_SUB=4 BUILD=build_exp LIBDIR=lib_exp`), kernel stats of kmeans_f32_probe.py each.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/kmf32_ab"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
P="$REPO/scripts/kmeans_f32_probe.py"
PKG="$REPO/event-camera-clustering-and-optical-flow-estimation_amd"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d "$OUT/a" -o a --output-format csv -- python3 "$P" 1 > "$OUT/a.log" 2>&1 || exit $?
ECC_LIB="$PKG/lib_exp/libecc.so" timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d "$OUT/b" -o b --output-format csv -- python3 "$P" 1 > "$OUT/b.log" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, sys, glob
out = sys.argv[1]
for tag in ("a", "b"):
    for r in csv.DictReader(open(glob.glob(f"{out}/{tag}/*kernel_stats.csv")[0])):
        print(tag, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
