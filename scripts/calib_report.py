#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE against known byte counts (scripts/calib/fetch_calib.hip).
Prints, per calibration kernel, the counter in bytes and its ratio to the bytes the kernel moves.
Usage: calib_report.py <evidence dir with calib_fetch/, calib_write/, calib_bytes.txt>"""
import csv
import glob
import re
import sys
from pathlib import Path


def counter(d, name):
    out = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != name:
                continue
            m = re.search(r"([A-Za-z_0-9]+(<[^>]*>)?)\(", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"]
            out[k] = out.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0
    return out


def main():
    d = sys.argv[1]
    known = {}
    for line in Path(d, "calib_bytes.txt").read_text().splitlines():
        name, b = line.rsplit(" ", 1)
        known[name.replace("unsigned int", "unsigned int")] = float(b)
    fetch, write = counter(d + "/calib_fetch", "FETCH_SIZE"), counter(d + "/calib_write", "WRITE_SIZE")
    print(f"{'kernel':28s} {'bytes':>12s} {'FETCH_SIZE':>12s} {'ratio':>6s} {'WRITE_SIZE':>12s} {'ratio':>6s}")
    for name, b in known.items():
        f = next((v for k, v in fetch.items() if k.replace("unsigned int", "uint32_t") == name or k == name), 0.0)
        w = next((v for k, v in write.items() if k == name), 0.0)
        print(f"{name:28s} {b:12.0f} {f:12.0f} {f / b:6.3f} {w:12.0f} {w / b:6.3f}")


if __name__ == "__main__":
    main()
