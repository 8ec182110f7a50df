"""BASELINE config C4 at full size inside the -m gpu suite: the bench's exact step — 20 004 864
synthetic events (1221 slices of 16384) on the 346x260 sensor, hash downsample in 8192-event
windows -> k-means k=16 (10 Lloyd passes + labels) on the representatives -> SAE + arc corners
with the per-slice 15x15 NMS in one call (ecc_fast_detect_nms) -> the corner tracker over all
1221 slices — against the oracle on the same events.

Reference path: DSA/metavision_sdk_get_started5_opencl_store.cpp:370-459 (downsample slices),
KM/assign_to_centers2.c:184-548 (k-means loop), FCT/metavision_time_surface_periodic_group_track.cpp
:815-1063 (SAE batch update, arc test, filterCorners, updateTrackedCorners per slice).

The oracle's stages run on the OpenMP restatement (oracle/cpu_omp.cpp, whose outputs the bench
checks equal to the 1-thread oracle) to keep this near one second of CPU; the tracker runs on the
1-thread oracle.  Bar: bit-exact everywhere (integer work, and the fp32 tracker in the reference's
operation order)."""
import numpy as np
import pytest

from parity import nms_mismatches, tracker_mismatches, windowed_mismatches

pytestmark = pytest.mark.gpu

W, H, SLICE, WINDOW, K, ITERS, CAP = 346, 260, 16384, 8192, 16, 10, 4096
N = 1221 * SLICE  # the bench's events per GPU per step


def test_c4_full_step_matches_oracle(ecc, orc, gpu):
    xy, t, _ = ecc.gen_events(N, seed=1, width=W, height=H)
    d_xy, d_t = ecc.DeviceArray.from_numpy(xy), ecc.DeviceArray.from_numpy(t)
    c0 = np.stack([np.linspace(20, W - 20, K), np.linspace(20, H - 20, K)[::-1]], 1).astype(np.float32).ravel()

    # ---- GPU: the bench's step (one stream)
    rep_xy, _, uniq, rep, nw = gpu.downsample_hash(d_xy, N, ecc.hash_cfg(window=WINDOW), want_idx=False)
    d_c = ecc.DeviceArray.from_numpy(c0)
    labels = ecc.DeviceArray(nw * WINDOW, np.uint8)
    gpu.kmeans_xy16_frame(rep_xy, nw, WINDOW, uniq, W, H, d_c, ecc.kmeans_cfg(k=K, max_iters=ITERS, tol=-1.0), labels)
    cfg = ecc.corner_cfg(width=W, height=H)
    sae = ecc.DeviceArray.zeros(W * H, np.int64)
    flags = ecc.DeviceArray(N, np.uint8)
    ns = N // SLICE
    out = ecc.DeviceArray(ns * CAP, ecc.CORNER_DTYPE)
    cnt = ecc.DeviceArray(ns, np.int32)
    gpu.fast_detect_nms(d_xy, d_t, N, cfg, sae, flags, 15, CAP, out, cnt)
    tr = ecc.Tracker(gpu)
    tr.update(out, cnt, ns, CAP)
    gpu.sync()
    assert gpu.fast_detect_status() == 0 and gpu.corner_nms_status() == 0 and tr.status() == 0
    stats = gpu.fast_detect_stats()
    g_tracks, g_groups = tr.tracks(), tr.groups()[0]
    tr.close()

    # ---- oracle
    o_rx, _, o_u, o_r = orc.omp_downsample_hash(xy, window=WINDOW)
    dense = np.concatenate([o_rx[w * WINDOW: w * WINDOW + o_u[w]] for w in range(len(o_u))])
    o_c, o_lab, _ = orc.omp_kmeans_run_xy16(dense, c0, ITERS)
    o_flags, o_sae = orc.omp_fast_detect(xy, t, W, H)
    o_out, o_cnt, _ = orc.omp_corner_nms(xy, o_flags, W, H, cap=CAP)
    otr = orc.OracleTracker(ecc.tracker_cfg())
    for s in range(ns):
        otr.update(o_out[s * CAP: s * CAP + o_cnt[s]])
    o_tracks, o_groups = otr.tracks(ecc.Track), otr.groups(ecc.Group)[0]

    # ---- bit-exact comparisons
    assert np.array_equal(uniq.numpy()[:nw], o_u) and np.array_equal(rep.numpy()[:nw], o_r)
    assert windowed_mismatches(rep_xy.numpy(), o_rx, o_u, WINDOW) == 0
    assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32))
    gl = labels.numpy()
    assert np.array_equal(np.concatenate([gl[w * WINDOW: w * WINDOW + o_u[w]] for w in range(nw)]), o_lab)
    g_flags = flags.numpy()
    assert int(o_flags.sum()) > 100_000  # the stream really has corners (592 930 at seed 1)
    bad = np.nonzero(g_flags != o_flags)[0]
    assert len(bad) == 0, (len(bad), bad[:8])
    assert np.array_equal(sae.numpy(), o_sae)
    assert np.array_equal(cnt.numpy(), o_cnt)
    assert nms_mismatches(out.numpy(), cnt.numpy(), o_out, o_cnt, CAP)[0] == 0
    assert len(o_tracks) > 0 and tracker_mismatches(g_tracks, o_tracks, g_groups, o_groups) == 0
    # the heavy windows went through arc_dense_kernel in this very run
    assert stats["overflow_items"] > 0 and stats["items"] == (ns + 31) // 32 * (-(-W // 14) * -(-H // 14))
