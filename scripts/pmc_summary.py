#!/usr/bin/env python3
"""Per-kernel SQ counters and occupancy from rocprofv3 --pmc passes (gpu_evidence.sh).

Occupancy follows rocprofiler-sdk's gfx950 definitions (counter_defs.yaml):
  MeanOccupancyPerCU = 4 * SQ_WAVE_CYCLES / max(GRBM_GUI_ACTIVE) / CU_NUM   (SQ_WAVE_CYCLES in quad-cycles)
  OccupancyPercent   = 100 * MeanOccupancyPerCU / 32                       (32 wave slots per CU)
rocprofv3's CSV sums GRBM_GUI_ACTIVE over the 8 XCD instances (measured: 7.8x the kernel's
duration in 2.4 GHz cycles for arc_kernel), so the per-instance value is the sum / 8.
Counters are summed per dispatch and averaged over a kernel's dispatches.
Usage: pmc_summary.py <dir with p*/ subdirs> <out.json> [n_cu] [n_xcd]
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from traffic import short  # noqa: E402


def main():
    d, out = sys.argv[1], sys.argv[2]
    n_cu = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    n_xcd = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    # (kernel, counter) -> {dispatch id: summed value}
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
        tag = Path(f).parts[len(Path(d).parts)]
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k.startswith("__amd"):
                continue
            per[(k, r["Counter_Name"])][(tag, r.get("Dispatch_Id", r.get("Correlation_Id", "0")))] += float(r["Counter_Value"])
    acc = defaultdict(dict)
    for (k, c), disp in per.items():
        acc[k][c] = sum(disp.values()) / max(len(disp), 1)
        acc[k]["dispatches"] = max(acc[k].get("dispatches", 0), len(disp))
    res = {}
    for k, c in sorted(acc.items()):
        row = {kk: (round(v, 1) if isinstance(v, float) else v) for kk, v in sorted(c.items())}
        g = c.get("GRBM_GUI_ACTIVE", 0.0) / n_xcd
        if g > 0:
            row["gpu_cycles"] = round(g)
        if g > 0 and "SQ_WAVE_CYCLES" in c:
            occ = 4.0 * c["SQ_WAVE_CYCLES"] / g / n_cu
            row["mean_waves_per_cu"] = round(occ, 2)
            row["occupancy_pct"] = round(100.0 * occ / 32.0, 1)
        if c.get("SQ_WAVE_CYCLES", 0) > 0:
            if "SQ_WAIT_ANY" in c:
                row["wait_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3)
            if "SQ_ACTIVE_INST_VALU" in c:
                row["valu_active_frac"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 3)
        if c.get("SQ_INSTS_LDS", 0) > 0 and "SQ_LDS_BANK_CONFLICT" in c:
            row["lds_conflict_cycles_per_inst"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"], 3)
        res[k] = row
    Path(out).write_text(json.dumps(res, indent=1))
    for k, r in res.items():
        if "occupancy_pct" in r:
            print(f"{k:28s} waves/CU {r['mean_waves_per_cu']:6.2f} ({r['occupancy_pct']:5.1f} %)  wait {r.get('wait_frac', 0):.2f}  "
                  f"valu {r.get('valu_active_frac', 0):.2f}")


if __name__ == "__main__":
    main()
