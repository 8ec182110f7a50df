#!/usr/bin/env python3
"""Per-kernel resource usage (VGPRs, spills, occupancy, LDS) of one HIP source.
Usage: kres.py <file.hip> [extra hipcc flags]"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
       "-fhip-fp32-correctly-rounded-divide-sqrt", *sys.argv[2:], "-c", sys.argv[1], "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = {}
for line in out.splitlines():
    m = re.search(r"remark: ([^:]+): (.*?) \[-R", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        continue
    cur[k] = v
    if k.startswith("LDS Size"):
        n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", cur["name"])[:64]
        print(f"{n:64s} vgpr={cur.get('VGPRs')} agpr={cur.get('AGPRs')} sgpr={cur.get('SGPRs')} "
              f"scratch={cur.get('ScratchSize [bytes/lane]')} occ={cur.get('Occupancy [waves/SIMD]')} lds={v}")
