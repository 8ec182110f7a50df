#!/bin/bash
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for d in 0 1 2 4; do
  OUT="$REPO/gpurun_out/pmc_dbg$d"; mkdir -p "$OUT"
  ECC_CORNER_DBG=$d timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d "$OUT" -o pmc --output-format csv -- python3 "$REPO/scripts/corner_probe.py" > "$OUT/probe.log" 2>&1 || exit $?
  f=$(find "$OUT" -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$d" <<'PY'
import csv, sys, collections, re
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "group_kernel" in r["Kernel_Name"]: acc[r["Counter_Name"]] += float(r["Counter_Value"])
print("dbg", sys.argv[2], {k: f"{v:.3g}" for k, v in sorted(acc.items())})
PY
  grep total "$OUT/probe.log" | cut -c1-80
done
