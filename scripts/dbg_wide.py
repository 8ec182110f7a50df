#!/usr/bin/env python3
"""Debug: the wide-time-range corner case (test_fast_detect_wide_time_ranges) with the library in
ECC_LIB, mismatch counts per case.  Usage: dbg_wide.py"""
import sys
from pathlib import Path
import numpy as np
R = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(R / "event-camera-clustering-and-optical-flow-estimation_amd"))
sys.path.insert(0, str(R / "oracle"))
import eccpy as ecc  # noqa: E402
import orc  # noqa: E402
gpu = ecc.Context(0)
W, H = 346, 260
for scale, jump in [(1000, 0), (1, 1 << 33), (300, 0), (97, 0), (1, 0)]:
    n = 16384 * 40 + 77
    xy, t, _ = ecc.gen_events(n, seed=41, width=W, height=H)
    t = t.astype(np.int64) * scale
    t[n // 3:] += jump
    o_flags, o_sae = orc.fast_detect(xy, t, W, H)
    for rep in range(2):
        cfg = ecc.corner_cfg(width=W, height=H)
        sae = ecc.DeviceArray.from_numpy(np.zeros(W * H, np.int64))
        flags = ecc.DeviceArray(n, np.uint8)
        gpu.fast_detect(ecc.DeviceArray.from_numpy(xy), ecc.DeviceArray.from_numpy(t), n, cfg, sae, flags)
        gpu.sync()
        g = flags.numpy()
        d = np.nonzero(g != o_flags)[0]
        print(scale, jump, rep, "oracle", int(o_flags.sum()), "gpu", int(g.sum()), "diff", len(d),
              "gpu-only", int(((g == 1) & (o_flags == 0)).sum()), "slices", np.unique(d // 16384)[:10], flush=True)
