#!/usr/bin/env python3
"""RAW ingest probe: the bench's events (20 M, 346x260) written as EVT 3.0 / EVT 2.0 words by the
library's RAW writer and decoded on the GPU; prints per-kernel times.  Usage: ingest_probe.py [n]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "event-camera-clustering-and-optical-flow-estimation_amd"))
import eccpy as ecc  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1221 * 16384
ctx = ecc.Context(0)
xy, t, p = ecc.gen_events(n, seed=1, width=346, height=260)
for fmt, name in ((ecc.EVT3, "EVT3"), (ecc.EVT2, "EVT2")):
    words = ecc.evt_encode(fmt, xy, t, p)
    dw = ecc.DeviceArray.from_numpy(words, ctx.stream)
    oxy, ot, op, on = (ecc.DeviceArray(n, np.uint32), ecc.DeviceArray(n, np.int64), ecc.DeviceArray(n, np.uint8),
                       ecc.DeviceArray(1, np.int64))
    ctx.set_timing(True)
    for rep in range(6):
        if rep == 1:
            ctx.timing_reset()
        ctx.evt_decode(fmt, dw, len(words), oxy, ot, op, n, on)
    st = ctx.timing_report()
    ctx.set_timing(False)
    print(name, len(words), "; ".join(f"{k} {1e3 * v['total_ms'] / v['launches']:.1f} us" for k, v in sorted(st.items())))
