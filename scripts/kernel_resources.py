#!/usr/bin/env python3
"""Per-kernel register, spill, scratch, LDS and occupancy table of libecc's HIP sources, as the
compiler reports them for gfx950 (-Rpass-analysis=kernel-resource-usage).  CPU only (hipcc
cross-compiles).  Usage: kernel_resources.py [source.hip ...] [--json out.json]

Occupancy [waves/SIMD] is the compiler's bound from VGPRs, SGPRs and LDS for the launch bounds;
bench.py's measured occupancy (SQ_WAVES / SQ_BUSY_CYCLES) is in profiles/<round>_occupancy.json.
"""
import json
import re
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent / "event-camera-clustering-and-optical-flow-estimation_amd"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-DECC_KM_ACC_SUB=4",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fvisibility=hidden", "-Rpass-analysis=kernel-resource-usage"]
FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "TotalSGPRs": "sgpr", "VGPRs Spill": "vgpr_spill", "SGPRs Spill": "sgpr_spill",
          "ScratchSize [bytes/lane]": "scratch_bytes_per_lane", "Occupancy [waves/SIMD]": "occupancy_waves_per_simd",
          "LDS Size [bytes/block]": "lds_bytes"}


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return out.stdout.split("\n")


def resources(src: Path):
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-c", str(src), "-o", "/dev/null"], capture_output=True, text=True)
    kernels, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"symbol": m.group(1), "source": src.name}
            kernels.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z][A-Za-z /\[\]]*?): (-?\d+)", line)
        if m and cur is not None and m.group(1) in FIELDS:
            cur[FIELDS[m.group(1)]] = int(m.group(2))
    names = demangle([k["symbol"] for k in kernels])
    for k, n in zip(kernels, names):
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        k["kernel"] = n.split("(")[0]
    return kernels


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    if out in args:
        args.remove(out)
    srcs = [Path(a) for a in args] or sorted((PKG / "csrc").glob("*.hip"))
    rows = [k for s in srcs for k in resources(s)]
    # rocPRIM's own sort kernels (sort.hip instantiates them): library code, not listed
    rows = [k for k in rows if "rocprim::" not in k["kernel"]]
    print(f"{'kernel':58s} {'vgpr':>4s} {'agpr':>4s} {'sgpr':>4s} {'vspill':>6s} {'scratch':>7s} {'lds':>6s} {'waves/SIMD':>10s}")
    for k in rows:
        print(f"{k['kernel'][:58]:58s} {k.get('vgpr', 0):4d} {k.get('agpr', 0):4d} {k.get('sgpr', 0):4d} "
              f"{k.get('vgpr_spill', 0):6d} {k.get('scratch_bytes_per_lane', 0):7d} {k.get('lds_bytes', 0):6d} "
              f"{k.get('occupancy_waves_per_simd', 0):10d}")
    if out:
        Path(out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
