#!/bin/bash
# SQ counters of the corner stage (corner_probe.py: fast_detect twice), three PMC passes of <= 8
# SQ counters each, no traces.  Prints per-kernel sums.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc2"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
P3="SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d "$OUT/p$i" -o p --output-format csv -- python3 "$REPO/scripts/corner_probe.py" > "$OUT/probe$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, sys, collections, re, glob
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"::([A-Za-z_0-9]+)(<[^>]*>)?\(", r["Kernel_Name"]); k = m.group(1) if m else r["Kernel_Name"][:30]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if k.startswith("__amd"): continue
    print(k); print("   ", {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
