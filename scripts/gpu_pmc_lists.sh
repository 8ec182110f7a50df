#!/bin/bash
# eps_lists / dbscan_extract: kernel stats, SQ counters and HBM traffic passes (eps_probe.py lists).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_lists"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
P="$REPO/scripts/eps_probe.py"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 "$P" lists > "$OUT/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 "$P" lists > "$OUT/write.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 "$P" lists > "$OUT/fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD -d "$OUT/sq" -o sq --output-format csv -- python3 "$P" lists > "$OUT/sq.log" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, sys, glob, collections
out = sys.argv[1]
for sub in ("write", "fetch", "sq"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for f in glob.glob(f"{out}/{sub}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        print(sub, k, {c: round(v / n[(k, c)]) for c, v in sorted(d.items())})
for r in csv.DictReader(open(glob.glob(out + "/trace/*kernel_stats.csv")[0])):
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
