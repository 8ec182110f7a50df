"""Pinning the oracle against the REFERENCE ITSELF: the reference's own OpenCL kernels
(coordinate_processor.cl, assign_to_centers.cl), compiled unmodified from /root/reference into
oracle/_ref/ by oracle/ref/Makefile, executed on the GPU box's OpenCL device by
oracle/ref/ref_harness.c.  Compares the reference kernel's outputs with the oracle (and so,
transitively, with the HIP path that test_gpu_parity.py checks against the oracle)."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REF = Path(__file__).resolve().parent.parent / "oracle" / "_ref"
HARNESS = REF / "ref_harness"


def _need_ref():
    if not HARNESS.exists():
        pytest.skip("oracle/_ref not built (reference tree absent where the repo was built)")


def _run(args, tmp_path):
    r = subprocess.run([str(HARNESS)] + [str(a) for a in args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


def _ref_downsample(tmp_path, pairs, lanes):
    (tmp_path / "in.i32").write_bytes(pairs.tobytes())
    _run(["downsample", REF / "coordinate_processor.gfx950.co", tmp_path / "in.i32", tmp_path / "out.i32", lanes], tmp_path)
    out = np.frombuffer((tmp_path / "out.i32").read_bytes(), np.int32)
    coords = out[2:].reshape(-1, 2)
    written = coords[(coords != -1).all(1)]
    return int(out[0]), int(out[1]), written


def _bucket(xx, yy):
    return (np.asarray(xx, np.int64) * 1619 + np.asarray(yy, np.int64) * 31) % 8192


@pytest.mark.parametrize("seed,n,wh", [(1, 8192, (346, 260)), (2, 8192, (1280, 720)), (3, 5000, (1400, 800)), (4, 1, (346, 260))])
def test_reference_process_coordinates_pins_oracle(ecc, orc, tmp_path, seed, n, wh):
    """One-wave launch: unique/repeated counts are final and must equal the oracle's.  The
    representative chosen per bucket is a race (Q2), so the reference's set of occupied buckets
    is compared and each of its representatives must be an event of that bucket."""
    _need_ref()
    xy, _, _ = ecc.gen_events(n, seed=seed, width=wh[0], height=wh[1])
    x, y = ecc.unpack_xy(xy)
    pairs = np.stack([x, y], 1).astype(np.int32)
    ref_unique, ref_repeated, ref_reps = _ref_downsample(tmp_path, pairs, 64)
    o_xy, o_idx, o_u, o_r = orc.downsample_hash(xy)
    assert ref_unique == o_u[0] and ref_repeated == o_r[0]
    assert len(ref_reps) == o_u[0]
    ox, oy = ecc.unpack_xy(o_xy[:o_u[0]])
    assert sorted(_bucket(ref_reps[:, 0], ref_reps[:, 1]).tolist()) == sorted(_bucket(ox, oy).tolist())
    valid = set(zip(x.tolist(), y.tolist()))
    assert all((int(a), int(b)) in valid for a, b in ref_reps)


def test_reference_process_coordinates_multiwave_race(ecc, orc, tmp_path):
    """Quirk Q21: with several waves (the reference launches 1024 lanes) lane 0 publishes the
    LDS counters before the other waves finish (no barrier, coordinate_processor.cl:80-81), so
    the reported counts can only UNDER-count; the coordinate list itself is still complete."""
    _need_ref()
    xy, _, _ = ecc.gen_events(8192, seed=1)
    x, y = ecc.unpack_xy(xy)
    pairs = np.stack([x, y], 1).astype(np.int32)
    ref_unique, ref_repeated, ref_reps = _ref_downsample(tmp_path, pairs, 256)
    _, _, o_u, o_r = orc.downsample_hash(xy)
    assert ref_unique <= o_u[0] and ref_repeated <= o_r[0]
    assert len(ref_reps) == o_u[0]


def test_reference_assign_to_centers_pins_oracle(ecc, orc, tmp_path):
    """assign_to_centers is deterministic: the reference kernel's label (2c or 255) must equal
    the oracle's (c or 255) for every point — pins the distance/threshold/tie semantics,
    including the device's OpenCL length() against IEEE sqrtf(dx*dx + dy*dy)."""
    _need_ref()
    rng = np.random.default_rng(7)
    cen = np.array([1, 1, 10, 10, 20, 20, 30, 30, 50, 50, 60, 60, 70, 70, 80, 80], np.float32)  # assign_to_centers2.c:131
    n = 256 * 400
    pts = np.concatenate([
        (np.arange(4096) % 100).astype(np.float32).reshape(-1, 2),        # the reference demo data (:123-129)
        rng.uniform(-30, 130, (n - 2048 - 4096, 2)).astype(np.float32),
        rng.integers(-20, 120, (4096, 2)).astype(np.float32),              # integer pixels: exact ties
    ])
    (tmp_path / "in.f32").write_bytes(pts.astype(np.float32).tobytes())
    (tmp_path / "c.f32").write_bytes(cen.tobytes())
    _run(["assign", REF / "assign_to_centers.gfx950.co", tmp_path / "in.f32", tmp_path / "c.f32", tmp_path / "out.i32"], tmp_path)
    ref = np.frombuffer((tmp_path / "out.i32").read_bytes(), np.int32)
    ref_lab = np.where(ref == 255, 255, ref // 2)
    o = orc.kmeans_assign_f32(pts.ravel(), cen).astype(np.int32)
    mism = np.nonzero(ref_lab != o)[0]
    assert len(mism) == 0, (len(mism), pts[mism[:5]], ref_lab[mism[:5]], o[mism[:5]])


def test_reference_kmeans_loop_pins_refcompat_oracle(orc, tmp_path):
    """The reference's three k-means kernels (assign_to_centers, assign_data_cluster,
    reduction_scalar) run on the GPU box's OpenCL device in the pass loop of
    KM/assign_to_centers2.c:184-548 (demo data, stale bins carried over, the y_offset index and
    int-abs update quirks Q7-Q9).  Each pass is replayed by orc_kmeans_refcompat_pass from the
    reference's own state before it (centroids, and the bin buffer read back in the previous
    pass: its stale tails depend on that pass's atomic order, Q8, so the oracle cannot predict
    them — it is given them): bin counts, the partial sums (per bin half: a bin above 1024 points
    splits between two 1024-float chunks in atomic order) and the updated centroids must be
    bit-identical in every pass (integer-valued floats < 2^24: every summation order is exact),
    and the restart decision must agree, so the oracle replays the whole run — whose length
    itself varies from run to run with the stale tails (scripts/kmeans_ref_debug.py prints it)."""
    _need_ref()
    out = tmp_path / "km.bin"
    _run(["kmeans_loop", REF / "assign_to_centers.gfx950.co", 50, out], tmp_path)
    raw = np.frombuffer(out.read_bytes(), np.int32)
    passes = int(raw[0])
    rec = raw[1:1 + 72 * passes].reshape(passes, 72)
    bufs = raw[1 + 72 * passes:].view(np.float32).reshape(passes, 8 * 4096)
    assert passes >= 2
    data = (np.arange(4096) % 100).astype(np.float32)
    c = np.array([1, 1, 10, 10, 20, 20, 30, 30, 50, 50, 60, 60, 70, 70, 80, 80], np.float32)
    buf = np.zeros(8 * 4096, np.float32)
    for k in range(passes):
        cnt = np.zeros(8, np.int32)
        ss = np.zeros(32, np.float32)
        again = orc.lib.orc_kmeans_refcompat_pass(data.ctypes.data, 2048, c.ctypes.data, buf.ctypes.data,
                                                  cnt.ctypes.data, ss.ctypes.data)
        assert np.array_equal(rec[k, :8], cnt), (k, rec[k, :8], cnt)
        # the sums enter the update only in (even, odd) chunk pairs = the x and y halves of a bin;
        # how a bin above 1024 points splits between its two chunks is the atomic order (Q8)
        r_ss = rec[k, 8:40].view(np.float32)
        assert np.array_equal(r_ss[0::2] + r_ss[1::2], ss[0::2] + ss[1::2]), (k, r_ss, ss)
        assert np.array_equal(rec[k, 56:72], c.view(np.int32)), (k, rec[k, 56:72].view(np.float32), c)
        assert again == (1 if k + 1 < passes else 0) or k + 1 == 50
        buf = bufs[k].copy()  # the reference's readback (its stale tails) for the next pass
