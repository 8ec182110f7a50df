#!/bin/bash
# SQ counters of the tracker kernel on the bench stream's corners (one --pmc pass each, no traces).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_tracker"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQC_ICACHE_MISSES SQC_ICACHE_HITS -d "$OUT/p1" -o p1 --output-format csv -- python3 "$REPO/scripts/tracker_probe.py" > "$OUT/p1.log" 2>&1; rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES -d "$OUT/p2" -o p2 --output-format csv -- python3 "$REPO/scripts/tracker_probe.py" > "$OUT/p2.log" 2>&1; rc=$?; echo "p2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "tracker" in r["Kernel_Name"]:
            kn = "fast" if "tracker_fast_kernel" in r["Kernel_Name"] else "general"
            acc[(kn, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (kn, k), v in sorted(acc.items()):
    print(f"{kn:8s} {k:24s} mean {sum(v)/len(v):14.1f}  n={len(v)}")
PY
