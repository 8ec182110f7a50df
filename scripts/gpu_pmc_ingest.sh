#!/bin/bash
# SQ counters for the RAW decoders (ingest_probe.py), one PMC pass.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_ingest"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM -d "$OUT" -o pmc --output-format csv -- python3 "$REPO/scripts/ingest_probe.py" > "$OUT/probe.log" 2>&1; rc=$?; echo "rc=$rc"
f=$(find "$OUT" -name "*counter_collection.csv" | head -1); echo "$f"
python3 - "$f" <<'PY'
import csv, sys, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"::([A-Za-z_0-9]+)(<[^>]*>)?\(", r["Kernel_Name"]); k = (m.group(0) if m else r["Kernel_Name"][:40])[:48]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print(k, {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
exit $rc
