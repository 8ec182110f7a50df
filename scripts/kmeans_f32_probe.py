#!/usr/bin/env python3
"""C3 f32 k-means probe (k=16, 50 M float points of 346x260 pixel coordinates, 10 Lloyd passes +
labels) for rocprofv3 counter passes.  Usage: kmeans_f32_probe.py [engine=1] [points=50e6]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "event-camera-clustering-and-optical-flow-estimation_amd"))
import eccpy as ecc  # noqa: E402

eng = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 50_000_000
W, H, K = 346, 260, 16
ctx = ecc.Context(0)
rng = np.random.default_rng(3)
f = np.empty(2 * n, np.float32)
f[0::2] = rng.integers(0, W, n)
f[1::2] = rng.integers(0, H, n)
d_f = ecc.DeviceArray.from_numpy(f, ctx.stream)
del f
c0 = np.stack([np.linspace(20, W - 20, K), np.linspace(20, H - 20, K)[::-1]], 1).astype(np.float32).ravel()
d_c0 = ecc.DeviceArray.from_numpy(c0, ctx.stream)
d_c = ecc.DeviceArray(2 * K, np.float32)
d_lab = ecc.DeviceArray(n, np.uint8)
for _ in range(2):
    ecc.check(ecc.lib.ecc_memcpy_d2d(d_c.ptr, d_c0.ptr, 8 * K, ctx.stream))
    ctx.kmeans_f32_engine(d_f, n, d_c, ecc.kmeans_cfg(k=K, max_iters=10, tol=-1.0), eng, d_lab)
ctx.sync()
print("ok", d_c.numpy()[:4], np.bincount(d_lab.numpy()[:1000000], minlength=17)[:4])
