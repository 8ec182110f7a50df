#!/usr/bin/env python3
"""Which matching paths of tracker_fast_kernel the dense parity cases take (profiling build:
make TRACKER_PROFILE=1 into another LIBDIR, selected by ECC_LIB).  Prints, per case, the
workgroup-wide rounds after round 0 and the one-wave tail rounds summed over the slices the fast
kernel ran, and the slice it handed over at (ctr->resume is not exported: a general-kernel
hand-over shows as fewer profiled slices)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "event-camera-clustering-and-optical-flow-estimation_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import eccpy as ecc  # noqa: E402
from test_gpu_parity import _dense_detections  # noqa: E402

cases = [(58, 120, 2, 4.0, {"max_frames": 2, "frames_to_skip": 1}),
         (59, 110, 40, 2.0, {"max_frames": 2, "frames_to_skip": 1, "max_distance": 12.0}),
         (53, 60, 4, 20.0, {"max_frames": 3, "frames_to_skip": 1, "history_size": 16, "group_radius": 40.0})]
ctx = ecc.Context(0)
prof = ecc.lib.ecc_tracker_profile
for seed, per, nc, spread, over in cases:
    dets = _dense_detections(seed, 36, per, nc, spread)
    cap = max(len(d) for d in dets)
    flat = np.zeros(36 * cap, ecc.CORNER_DTYPE)
    cnt = np.zeros(36, np.int32)
    for s, d in enumerate(dets):
        flat[s * cap: s * cap + len(d)] = d
        cnt[s] = len(d)
    tr = ecc.Tracker(ctx, ecc.tracker_cfg(**over))
    tr.update(ecc.DeviceArray.from_numpy(flat), ecc.DeviceArray.from_numpy(cnt), 36, cap)
    ctx.sync()
    o, tpu = (C.c_ulonglong * 16)(), C.c_double()
    prof(o, C.byref(tpu))
    print(f"seed {seed}: max C {cnt.max()}, workgroup rounds after round 0 {o[6] - 36}, tail rounds {o[9]}, "
          f"tracks {len(tr.tracks())}", flush=True)
