#!/bin/bash
# SQ counter passes over the eps kernels (eps_probe.py).  Usage: gpu_pmc_eps.sh [what]
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_eps"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
W="${1:-all}"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 "$REPO/scripts/eps_probe.py" "$W" > "$OUT/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d "$OUT/sq" -o sq --output-format csv -- python3 "$REPO/scripts/eps_probe.py" "$W" > "$OUT/sq.log" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, sys, glob, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(glob.glob(out + "/sq/*counter_collection.csv")[0])):
    k = r["Kernel_Name"].split("(")[0][-48:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / n[(k, c)]) for c, v in sorted(d.items())})
for r in csv.DictReader(open(glob.glob(out + "/trace/*kernel_stats.csv")[0])):
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
