#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KiB per dispatch).

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports exactly half of the bytes
of wide coalesced streaming reads, so reads are doubled; WRITE_SIZE is exact for 16-B/lane
streaming stores.  Other access patterns are uncalibrated — reported as-is in the raw fields.
Usage: traffic.py <prof_dir> <out.json>
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    m = re.search(r"::([A-Za-z_0-9]+)(<[^>]*>)?\(", name)
    base = m.group(1) if m else name.split("(")[0]
    # map to the names libecc's timing report (and bench.py) use
    if base in ("kmeans_xy16_kernel", "kmeans_fast_kernel"):
        return "kmeans_xy16_labels" if re.search(r"<(\d+, )?false[,>]", name) else "kmeans_xy16_kernel"
    if base in ("kmeans_lds_labels_kernel", "kmeans_img_labels_kernel"):
        return "kmeans_xy16_labels"
    if base in ("nms_grid_kernel", "nms_greedy_kernel"):
        return "nms_kernel"
    if base == "kmeans_step_kernel" and re.search(r"<\d+, true>", name):
        return "kmeans_pixel_pass"
    if base == "flags_event_kernel":
        return "flags_kernel"
    return base


def load(path, counter):
    acc = defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        acc[k][0] += float(r["Counter_Value"]) * 1024.0
        acc[k][1] += 1
    return acc


def main():
    d = Path(sys.argv[1])
    fetch = load(next(d.glob("fetch/*counter_collection.csv")), "FETCH_SIZE")
    write = load(next(d.glob("write/*counter_collection.csv")), "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        fb, fn = fetch.get(k, [0.0, 1])
        wb, wn = write.get(k, [0.0, 1])
        f, w = fb / max(fn, 1), wb / max(wn, 1)
        out[k] = {"bytes_per_launch": 2 * f + w, "fetch_raw_per_launch": f, "write_per_launch": w,
                  "launches": fn, "correction": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halves wide reads)"}
    Path(sys.argv[2]).write_text(json.dumps(out, indent=1))
    for k, v in out.items():
        print(f"{k:28s} {v['bytes_per_launch']/1e6:10.3f} MB/launch  (fetch raw {v['fetch_raw_per_launch']/1e6:.3f}, write {v['write_per_launch']/1e6:.3f})")


if __name__ == "__main__":
    main()
