#!/usr/bin/env python3
"""Replays the reference k-means loop (oracle/_ref/ref_harness kmeans_loop) pass by pass with
orc_kmeans_refcompat_pass from the reference's own state; prints per pass the bin counts, any
half-bin sum difference and how far the oracle's bin buffer differs from the reference's readback
(positions differ by atomic order — Q8 — only the sums matter).  GPU box only."""
import sys, subprocess, numpy as np
sys.path.insert(0, 'oracle'); import orc
subprocess.run(["oracle/_ref/ref_harness", "kmeans_loop", "oracle/_ref/assign_to_centers.gfx950.co", "50", "gpurun_out/km.bin"], check=True)
raw = np.fromfile("gpurun_out/km.bin", np.int32)
passes = int(raw[0]); rec = raw[1:1+72*passes].reshape(passes, 72); bufs = raw[1+72*passes:].view(np.float32).reshape(passes, -1)
data = (np.arange(4096) % 100).astype(np.float32)
c = np.array([1,1,10,10,20,20,30,30,50,50,60,60,70,70,80,80], np.float32)
buf = np.zeros(8*4096, np.float32)
for k in range(passes):
    cnt = np.zeros(8, np.int32); ss = np.zeros(32, np.float32); cb = c.copy(); bb = buf.copy()
    again = orc.lib.orc_kmeans_refcompat_pass(data.ctypes.data, 2048, c.ctypes.data, bb.ctypes.data, cnt.ctypes.data, ss.ctypes.data)
    rs = rec[k, 8:40].view(np.float32)
    rs, ss = rs[0::2] + rs[1::2], ss[0::2] + ss[1::2]
    print(k, "cnt", rec[k,:8].tolist(), cnt.tolist())
    d = np.nonzero(rs != ss)[0]
    print("  ss diff idx", d.tolist(), rs[d].tolist(), ss[d].tolist())
    # compare buffers: oracle's bb vs ref's bufs[k]
    bd = np.nonzero(bb != bufs[k])[0]
    print("  buf diffs", len(bd), bd[:10].tolist(), bb[bd[:10]].tolist(), bufs[k][bd[:10]].tolist())
    if len(d): break
    buf = bufs[k].copy()
