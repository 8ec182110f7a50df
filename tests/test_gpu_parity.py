"""GPU parity tests: every HIP entry point through the C ABI against the oracle (CPU restatement)
on the same seeded inputs.  Bar: bit-exact for integer / index / label work and for the fp32
tracker (identical operation order), 1e-4 for float-input k-means centroids."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W_SMALL, H_SMALL = 346, 260


def dev(ecc, a):
    return ecc.DeviceArray.from_numpy(np.ascontiguousarray(a))


# ------------------------------------------------------------------------------ numerics
def test_device_sqrt_is_correctly_rounded(ecc, gpu):
    """ecc::sqrt_rn (used by k-means, tracker) == IEEE sqrtf for random and edge inputs."""
    rng = np.random.default_rng(0)
    parts = [rng.uniform(0, 1e5, 2_000_000), rng.integers(0, 1 << 20, 1_000_000),
             np.exp(rng.uniform(-80, 80, 1_000_000)), (np.arange(1, 200000) ** 2),
             np.array([0.0, np.inf, 1e-40, 1e-45, 2.0 ** -100, 3.4e38])]
    x = np.concatenate([p.astype(np.float32) for p in parts])
    # also the neighbours of exact squares (where rounding decisions are tight)
    sq = (np.arange(1, 100000, dtype=np.float32) ** 2)
    x = np.concatenate([x, np.nextafter(sq, np.float32(np.inf)), np.nextafter(sq, np.float32(0))]).astype(np.float32)
    d_in = dev(ecc, x)
    d_out = ecc.DeviceArray(len(x), np.float32)
    ecc.check(ecc.lib.ecc_util_sqrt_f32(gpu.ctx, d_in.ptr, d_out.ptr, len(x), gpu.stream))
    gpu.sync()
    got = d_out.numpy()
    ref = np.sqrt(x)
    bad = np.nonzero(got.view(np.uint32) != ref.view(np.uint32))[0]
    assert len(bad) == 0, (x[bad[:5]], got[bad[:5]], ref[bad[:5]])


# ------------------------------------------------------------------------------ downsample
@pytest.mark.parametrize("n,window,seed,wh", [
    (200_000, 8192, 1, (346, 260)),
    (123_457, 8192, 2, (1280, 720)),
    (50_001, 1000, 3, (1280, 720)),      # ragged last window, window not a multiple of 1024
    (70_000, 16384, 4, (346, 260)),
    (8192, 8192, 5, (1400, 800)),        # coordinates beyond the inclusive 1280/720 bounds (:56)
    (1, 8192, 6, (346, 260)),
])
def test_downsample_matches_oracle(ecc, orc, gpu, n, window, seed, wh):
    xy, _, _ = ecc.gen_events(n, seed=seed, width=wh[0], height=wh[1])
    cfg = ecc.hash_cfg(window=window)
    d_xy = dev(ecc, xy)
    rep_xy, rep_idx, uniq, rep, nw = gpu.downsample_hash(d_xy, n, cfg)
    gpu.sync()
    o_xy, o_idx, o_u, o_r = orc.downsample_hash(xy, window=window)
    g_u, g_r = uniq.numpy()[:nw], rep.numpy()[:nw]
    assert (g_u == o_u).all() and (g_r == o_r).all()
    gx, gi = rep_xy.numpy(), rep_idx.numpy()
    for w in range(nw):
        k = o_u[w]
        sl = slice(w * window, w * window + k)
        assert (gx[sl] == o_xy[sl]).all(), f"window {w} representatives differ"
        assert (gi[sl] == o_idx[sl]).all(), f"window {w} representative indices differ"


@pytest.mark.parametrize("n,window,wh,seed", [(8192 * 5 + 77, 8192, (346, 260), 3), (50_000, 8192, (1280, 720), 4),
                                              (20_000, 1000, (40, 30), 5), (1, 8192, (346, 260), 6)])
def test_dedup_exact_matches_oracle(ecc, orc, gpu, n, window, wh, seed):
    """analyzeCoordinates (a4): unique counts, first-occurrence order and per-coordinate counts;
    (40, 30) packs each window with many repeats of few coordinates."""
    xy, _, _ = ecc.gen_events(n, seed=seed, width=wh[0], height=wh[1])
    g_idx, g_cnt, g_u, nw = gpu.dedup_exact(dev(ecc, xy), n, window)
    gpu.sync()
    o_idx, o_cnt, o_u = orc.dedup_exact(xy, window)
    assert (g_u.numpy()[:nw] == o_u).all()
    gi, gc = g_idx.numpy(), g_cnt.numpy()
    for w in range(nw):
        sl = slice(w * window, w * window + o_u[w])
        assert (gi[sl] == o_idx[sl]).all() and (gc[sl] == o_cnt[sl]).all()
        assert gc[sl].sum() == min(window, n - w * window)


@pytest.mark.parametrize("wh", [(1280, 720), (346, 260)])
def test_downsample_full_size_properties(ecc, gpu, wh):
    """10 M events (BASELINE config C2, both sensors) — size-independent properties: every
    representative is the first event of its bucket, buckets are distinct, counts agree with
    the outputs."""
    n = 10_000_000
    xy, _, _ = ecc.gen_events(n, seed=11, width=wh[0], height=wh[1])
    d_xy = dev(ecc, xy)
    rep_xy, rep_idx, uniq, rep, nw = gpu.downsample_hash(d_xy, n)
    gpu.sync()
    u, r, rx, ri = uniq.numpy(), rep.numpy(), rep_xy.numpy(), rep_idx.numpy()
    assert nw == 1221 and (u <= 8192).all() and (r <= u).all()
    rng = np.random.default_rng(0)
    for w in rng.choice(nw, 24, replace=False):
        lo = w * 8192
        ev = xy[lo:lo + 8192]
        x, y = ev & 0xFFFF, ev >> 16
        h = (x.astype(np.int64) * 1619 + y.astype(np.int64) * 31) % 8192
        first = {}
        cnt = {}
        for i, b in enumerate(h):
            first.setdefault(int(b), i)
            cnt[int(b)] = cnt.get(int(b), 0) + 1
        k = u[w]
        assert k == len(first) and r[w] == sum(1 for c in cnt.values() if c >= 2)
        exp_idx = np.array(sorted(first.values()), np.int64) + lo
        assert (ri[lo:lo + k] == exp_idx).all()
        assert (rx[lo:lo + k] == xy[exp_idx]).all()


# ------------------------------------------------------------------------------ k-means
def _reps(ecc, orc, n=400_000, seed=7):
    xy, _, _ = ecc.gen_events(n, seed=seed)
    o_xy, _, o_u, _ = orc.downsample_hash(xy)
    return xy, o_xy, o_u


def _init_centroids(k, seed=0, w=W_SMALL, h=H_SMALL):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(0, w, k), rng.uniform(0, h, k)], 1).astype(np.float32).ravel()


@pytest.mark.parametrize("k,iters,tol", [(16, 10, -1.0), (8, 20, 1e-3), (64, 3, -1.0), (1, 4, -1.0)])
def test_kmeans_xy16_segmented_matches_oracle(ecc, orc, gpu, k, iters, tol):
    xy, rep_xy, u = _reps(ecc, orc)
    nw = len(u)
    dense = np.concatenate([rep_xy[w * 8192: w * 8192 + u[w]] for w in range(nw)])
    c0 = _init_centroids(k)
    o_c, o_lab, o_it = orc.kmeans_run_xy16(dense, c0, iters, 50.0, tol)
    d_rep = dev(ecc, rep_xy)
    d_cnt = dev(ecc, u)
    d_c = dev(ecc, c0)
    d_lab = ecc.DeviceArray(len(rep_xy), np.uint8)
    d_it = ecc.DeviceArray(1, np.int32)
    cfg = ecc.kmeans_cfg(k=k, max_iters=iters, tol=tol)
    gpu.kmeans_xy16(d_rep, nw, 8192, d_cnt, d_c, cfg, d_lab, d_it)
    gpu.sync()
    g_c = d_c.numpy()
    assert d_it.numpy()[0] == o_it
    assert np.array_equal(g_c.view(np.uint32), o_c.view(np.uint32)), (g_c, o_c)
    g_lab = d_lab.numpy()
    g_dense = np.concatenate([g_lab[w * 8192: w * 8192 + u[w]] for w in range(nw)])
    assert (g_dense == o_lab).all()


def test_kmeans_xy16_dense_matches_oracle(ecc, orc, gpu):
    xy, _, _ = ecc.gen_events(300_001, seed=9)
    c0 = _init_centroids(16, 3)
    o_c, o_lab, o_it = orc.kmeans_run_xy16(xy, c0, 6)
    d_c = dev(ecc, c0)
    d_lab = ecc.DeviceArray(len(xy), np.uint8)
    gpu.kmeans_xy16(dev(ecc, xy), 1, len(xy), None, d_c, ecc.kmeans_cfg(k=16, max_iters=6, tol=-1.0), d_lab)
    gpu.sync()
    assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32))
    assert (d_lab.numpy() == o_lab).all()


@pytest.mark.parametrize("k", [16, 24, 40])
def test_kmeans_xy16_ties_take_exact_path(ecc, orc, gpu, k):
    """Each centre has an EARLIER twin one ulp to its right: for points roughly above/below the
    pair, the twin's d2 is a few ulps larger (the fast kernel's near-tie branch, ~25% of points)
    and in ~4% the two square roots round equal, so the reference picks the earlier twin despite
    its larger d2.  k=24 uses the K=32 instance, k=40 the generic kernel."""
    rng = np.random.default_rng(k)
    n = 200_003
    half = k // 2
    cx = rng.integers(20, 320, half).astype(np.float32) + np.float32(0.25)
    cy = rng.integers(20, 240, half).astype(np.float32)
    c0 = np.empty((k, 2), np.float32)
    c0[:half, 0], c0[:half, 1] = np.nextafter(cx, np.float32(np.inf)), cy
    c0[half:2 * half, 0], c0[half:2 * half, 1] = cx, cy
    if k % 2:
        c0[-1] = c0[0]
    c0 = c0.ravel()
    ci = rng.integers(0, half, n)
    x = np.clip(np.round(cx[ci] + rng.normal(0, 2, n)), 0, 345).astype(np.int64)
    y = np.clip(np.round(cy[ci] + rng.normal(0, 25, n)), 0, 259).astype(np.int64)
    xy = ecc.pack_xy(x, y)
    o_c, o_lab, o_it = orc.kmeans_run_xy16(xy, c0, 2, 50.0, -1.0)
    d_c = dev(ecc, c0)
    d_lab = ecc.DeviceArray(n, np.uint8)
    gpu.kmeans_xy16(dev(ecc, xy), 1, n, None, d_c, ecc.kmeans_cfg(k=k, max_iters=2, tol=-1.0), d_lab)
    gpu.sync()
    assert (d_lab.numpy() == o_lab).all()
    assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32))


@pytest.mark.parametrize("k", [16, 32])
def test_kmeans_xy16_points_outside_pixel_grid(ecc, orc, gpu, k):
    """Coordinates up to 6000 x 3000: the pixel-histogram path sends the points beyond its
    2048 x 2048 grid through the overflow list; results must not change."""
    rng = np.random.default_rng(77 + k)
    n = 300_007
    x = np.concatenate([rng.integers(0, 6000, n // 2), rng.normal(700, 80, n - n // 2).clip(0, 65535)]).astype(np.int64)
    y = np.concatenate([rng.integers(0, 3000, n // 2), rng.normal(400, 60, n - n // 2).clip(0, 65535)]).astype(np.int64)
    xy = ecc.pack_xy(x, y)
    c0 = np.stack([rng.uniform(0, 6000, k), rng.uniform(0, 3000, k)], 1).astype(np.float32).ravel()
    o_c, o_lab, o_it = orc.kmeans_run_xy16(xy, c0, 5, 3000.0, -1.0)
    d_c = dev(ecc, c0)
    d_lab = ecc.DeviceArray(n, np.uint8)
    gpu.kmeans_xy16(dev(ecc, xy), 1, n, None, d_c, ecc.kmeans_cfg(k=k, max_iters=5, tol=-1.0, threshold=3000.0), d_lab)
    gpu.sync()
    assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32))
    assert (d_lab.numpy() == o_lab).all()


def test_kmeans_f32_matches_oracle(ecc, orc, gpu):
    rng = np.random.default_rng(5)
    pts = np.concatenate([rng.normal(m, 6.0, (20000, 2)) for m in ([40, 40], [120, 60], [200, 180], [300, 90])])
    pts = pts.astype(np.float32).ravel()
    c0 = np.array([30, 30, 110, 70, 210, 170, 290, 100], np.float32)
    o_c, o_lab, _ = orc.kmeans_run_f32(pts, c0, 8)
    d_c = dev(ecc, c0)
    d_lab = ecc.DeviceArray(len(pts) // 2, np.uint8)
    gpu.kmeans_f32(dev(ecc, pts), len(pts) // 2, d_c, ecc.kmeans_cfg(k=4, max_iters=8, tol=-1.0), d_lab)
    gpu.sync()
    assert np.allclose(d_c.numpy(), o_c, atol=1e-4, rtol=0)   # north_star tolerance for centroids
    assert (d_lab.numpy() != o_lab).mean() < 1e-4


@pytest.mark.parametrize("engine", [1, 2, 3])
@pytest.mark.parametrize("k,data", [(16, "float"), (5, "int"), (32, "int"), (16, "ties")])
def test_kmeans_f32_engines_match_oracle(ecc, orc, gpu, engine, k, data):
    """Both assignment engines (vector / matrix cores): labels identical to the oracle's
    assign_to_centers rule; centroids bit-exact for integer-valued points (fp64 sums are exact),
    within 1e-4 otherwise.  'ties': points on a small integer grid with coinciding centres, so the
    matrix engine's exact fallback decides most points."""
    rng = np.random.default_rng(k * 7 + engine)
    if data == "float":
        pts = np.concatenate([rng.normal(m, 9.0, (40000, 2)) for m in rng.uniform(0, 340, (8, 2))])
    elif data == "int":
        pts = np.floor(rng.uniform(0, 346, (300001, 2)))
    else:
        pts = rng.integers(0, 12, (100000, 2)).astype(np.float64)
    pts = pts.astype(np.float32).ravel()
    if data == "ties":
        c0 = np.array([[3, 3], [3, 3], [8, 8], [3, 8], [8, 3]] * 4, np.float32)[:k].ravel()
    else:
        c0 = _init_centroids(k, seed=k)
    iters = 5
    o_c, o_lab, o_it = orc.kmeans_run_f32(pts, c0, iters)
    d_c = dev(ecc, c0)
    d_lab = ecc.DeviceArray(len(pts) // 2, np.uint8)
    d_it = ecc.DeviceArray(1, np.int32)
    gpu.kmeans_f32_engine(dev(ecc, pts), len(pts) // 2, d_c, ecc.kmeans_cfg(k=k, max_iters=iters, tol=-1.0), engine,
                          d_lab, d_it)
    gpu.sync()
    g_c = d_c.numpy()
    assert d_it.numpy()[0] == o_it
    if data == "float":
        assert np.allclose(g_c, o_c, atol=1e-4, rtol=0)
        assert (d_lab.numpy() != o_lab).mean() < 1e-4
    else:
        assert np.array_equal(g_c.view(np.uint32), o_c.view(np.uint32)), (g_c, o_c)
        assert (d_lab.numpy() == o_lab).all()


def test_kmeans_assign_ties_and_threshold(ecc, orc, gpu):
    """assign_to_centers semantics: first minimum wins, strict < threshold 50, 255 = none."""
    c = np.array([10, 10, 20, 10, 10, 10, 100, 100], np.float32)  # centres 0 and 2 coincide
    pts = np.array([[15, 10], [10, 10], [60, 10], [59.99, 10], [100, 149.99], [100, 150], [17.5, 10]], np.float32)
    rng = np.random.default_rng(1)
    pts = np.concatenate([pts, rng.uniform(-20, 200, (100000, 2)).astype(np.float32)]).ravel()
    o = orc.kmeans_assign_f32(pts, c)
    d_lab = ecc.DeviceArray(len(pts) // 2, np.uint8)
    gpu.kmeans_assign_f32(dev(ecc, pts), len(pts) // 2, dev(ecc, c), 4, 50.0, d_lab)
    gpu.sync()
    g = d_lab.numpy()
    assert (g == o).all()
    assert list(g[:7]) == [0, 0, 1, 1, 3, 255, 1]


@pytest.mark.parametrize("engine", [1, 2, 3])
def test_kmeans_f32_threshold_and_tie_boundaries_ulps(ecc, orc, gpu, engine):
    """The f32 engines' fast screens (the vector engine's 32-ulp buckets + d2 < thr2, the matrix
    engine's margin) against assign_to_centers' rule at its edges: points a few ulps either side
    of the threshold circle (sqrt(d2) < 50) and of the bisector between two centres."""
    rng = np.random.default_rng(17 + engine)
    c = np.array([100, 100, 180, 100, 100, 180, 35.5, 41.25], np.float32)
    th = rng.uniform(0, 2 * np.pi, 60000)
    ring = np.stack([100 + 50 * np.cos(th), 100 + 50 * np.sin(th)], 1).astype(np.float32)
    bis = np.stack([np.full(60000, 140.0), rng.uniform(60, 140, 60000)], 1).astype(np.float32)
    pts = np.concatenate([ring, bis])
    steps = rng.integers(-4, 5, pts.shape).astype(np.int32)
    pts = (pts.view(np.int32) + steps).view(np.float32)  # +-4 ulps
    flat = pts.ravel()
    o = orc.kmeans_assign_f32(flat, c)
    assert 0 < (o == 255).sum() < len(o) and (o == 1).sum() > 1000
    d_c = dev(ecc, c)
    d_lab = ecc.DeviceArray(len(pts), np.uint8)
    gpu.kmeans_f32_engine(dev(ecc, flat), len(pts), d_c, ecc.kmeans_cfg(k=4, max_iters=0, tol=-1.0), engine, d_lab)
    gpu.sync()
    assert (d_lab.numpy() == o).all()


@pytest.mark.parametrize("case", ["stacked", "outliers", "tiny", "far", "converge"])
def test_kmeans_f32_candidate_table_edges(ecc, orc, gpu, case):
    """The vector engine's candidate table (64 x 64 cells over a sampled bounding box, <= 3
    candidates per cell): labels and centroids equal the oracle's where the table's cases meet —
    five coinciding centres (cells with > 3 candidates), a few points far outside the sampled box
    plus NaN / inf points, a sub-pixel extent (the minimum cell size), every cell beyond the
    threshold, and a run that converges on tol (the table of the converging update is the one the
    labels use)."""
    rng = np.random.default_rng({"stacked": 1, "outliers": 2, "tiny": 3, "far": 4, "converge": 5}[case])
    n = 400_000
    pts = np.floor(rng.uniform(0, 346, (n, 2))).astype(np.float32)
    c0 = _init_centroids(16, seed=21, w=346, h=260)
    iters, tol, thr, exact = 4, -1.0, 50.0, True
    if case == "stacked":
        c0.reshape(-1, 2)[3:8] = [120.0, 90.0]  # five centres on one point: > 3 candidates nearby
        c0.reshape(-1, 2)[8:10] = [121.0, 90.0]
    elif case == "outliers":
        pts[rng.integers(0, n, 40)] = rng.uniform(-3e4, 3e4, (40, 2))
    elif case == "tiny":
        pts = (100.0 + rng.uniform(0, 1e-3, (n, 2))).astype(np.float32)
        c0 = (100.0 + rng.uniform(0, 1e-3, (16, 2))).astype(np.float32).ravel()
        exact = False
    elif case == "far":
        thr = 0.25  # most cells hold no point within the threshold of any centre
    else:
        iters, tol = 40, 0.05
    flat = pts.ravel()
    o_c, o_lab, o_it = orc.kmeans_run_f32(flat, c0, iters, thr, tol)
    d_c, d_lab, d_it = dev(ecc, c0), ecc.DeviceArray(n, np.uint8), ecc.DeviceArray(1, np.int32)
    gpu.kmeans_f32_engine(dev(ecc, flat), n, d_c, ecc.kmeans_cfg(k=16, max_iters=iters, tol=tol, threshold=thr), 1,
                          d_lab, d_it)
    gpu.sync()
    assert d_it.numpy()[0] == o_it
    if exact:  # integer-valued points: fp64 sums exact, centroids bit-equal
        assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32))
        assert (d_lab.numpy() == o_lab).all()
    else:
        assert np.allclose(d_c.numpy(), o_c, atol=1e-6, rtol=0)
        assert (d_lab.numpy() != o_lab).mean() < 1e-4
    # labels of non-finite points with the final centres (labels-only pass, max_iters 0)
    bad = pts[:1000].copy()
    bad[::7, 0] = np.nan
    bad[1::7, 1] = np.inf
    bad[2::7] = -np.inf
    d_lab2 = ecc.DeviceArray(len(bad), np.uint8)
    gpu.kmeans_f32_engine(dev(ecc, bad.ravel()), len(bad), d_c, ecc.kmeans_cfg(k=16, max_iters=0, threshold=thr), 1,
                          d_lab2)
    gpu.sync()
    assert (d_lab2.numpy() == orc.kmeans_assign_f32(bad.ravel(), d_c.numpy(), thr)).all()


@pytest.mark.parametrize("engine", [2, 3])
@pytest.mark.parametrize("k", [1, 3, 16])
def test_kmeans_f32_matrix_engines_extreme_points(ecc, orc, gpu, engine, k):
    """The matrix engines' margin screen on the points it must hand to the exact path: NaN, +-inf,
    huge (|p| 1e19..1e30: infinite or NaN MFMA values), subnormal and negative coordinates, an odd
    point count; labels-only pass against assign_to_centers.  (Found: the unused centre slots of
    k < 16 were padded with 1e30, which a point at (1e30, 1e30) matched exactly; they are +inf now,
    never within any threshold.)"""
    rng = np.random.default_rng(40 + engine + k)
    pts = rng.uniform(-50, 400, (20001, 2)).astype(np.float32)
    pts[::11, 0] = np.nan
    pts[1::11, 1] = np.inf
    pts[2::11] = -np.inf
    pts[3::11] = rng.choice([1e19, -1e19, 1e30, -3e30], (len(pts[3::11]), 2))
    pts[4::11] = rng.choice([1e-40, -1e-41, 0.0, -0.0], (len(pts[4::11]), 2))
    c = rng.uniform(-20, 380, (k, 2)).astype(np.float32)
    c[0] = [0.0, 0.0]
    flat = pts.ravel()
    d_lab = ecc.DeviceArray(len(pts), np.uint8)
    for thr in (50.0, 1e35):
        gpu.kmeans_f32_engine(dev(ecc, flat), len(pts), dev(ecc, c.ravel()),
                              ecc.kmeans_cfg(k=k, max_iters=0, tol=-1.0, threshold=thr), engine, d_lab)
        gpu.sync()
        g, o = d_lab.numpy(), orc.kmeans_assign_f32(flat, c.ravel(), thr)
        bad = np.flatnonzero(g != o)
        assert len(bad) == 0, (thr, len(bad), [(pts[i].tolist(), int(g[i]), int(o[i])) for i in bad[:6]], c.tolist())


@pytest.mark.parametrize("engine", [1, 2, 3])
def test_kmeans_f32_engines_subnormal_squares(ecc, orc, gpu, engine):
    """Points and centres around 1e-20: every |c|^2, |p|^2 and d^2 is subnormal in fp32, so a
    flush-to-zero anywhere in the screen (the matrix engines' |c|^2 - 2 c.p products, the vector
    engine's table) would tie centres the reference (`length()` with IEEE subnormals,
    assign_to_centers.cl:15-25) tells apart.  The engines' margin argument assumes only that each
    rounding is bounded, not the order in which the matrix core sums the products; the exact
    fallback must catch every point the screen cannot decide.  Labels-only passes at three
    thresholds against the oracle's assignment."""
    rng = np.random.default_rng(90 + engine)
    pts = (rng.uniform(-3.0, 3.0, (30001, 2)) * 1e-20).astype(np.float32)
    pts[::13] = (rng.integers(-3, 4, (len(pts[::13]), 2)) * 1e-20).astype(np.float32)  # ties
    c = (rng.uniform(-2.5, 2.5, (16, 2)) * 1e-20).astype(np.float32)
    flat = pts.ravel()
    d_lab = ecc.DeviceArray(len(pts), np.uint8)
    for thr in (50.0, 2e-20, 7e-21):
        gpu.kmeans_f32_engine(dev(ecc, flat), len(pts), dev(ecc, c.ravel()),
                              ecc.kmeans_cfg(k=16, max_iters=0, tol=-1.0, threshold=thr), engine, d_lab)
        gpu.sync()
        g, o = d_lab.numpy(), orc.kmeans_assign_f32(flat, c.ravel(), thr)
        bad = np.flatnonzero(g != o)
        assert len(bad) == 0, (thr, len(bad), [(pts[i].tolist(), int(g[i]), int(o[i])) for i in bad[:6]])
        assert len(set(o.tolist())) > 8  # the case really separates many centres


# ------------------------------------------------------------------------------ SAE + arc corners
def _fast_gpu(ecc, gpu, xy, t, W, H, border_mode=0, first_detect=1, sae0=None, slice_events=16384):
    cfg = ecc.corner_cfg(width=W, height=H, border_mode=border_mode, first_detect_slice=first_detect,
                         slice_events=slice_events)
    sae = dev(ecc, np.zeros(W * H, np.int64) if sae0 is None else sae0)
    flags = ecc.DeviceArray(len(xy), np.uint8)
    gpu.fast_detect(dev(ecc, xy), dev(ecc, t), len(xy), cfg, sae, flags)
    assert gpu.fast_detect_status() == 0
    return flags.numpy(), sae.numpy()


@pytest.mark.parametrize("scale,jump", [
    (1000, 0),        # ns ticks: a group spans > 2^27 ticks (arc staging takes the int64 clamp path)
    (1, 1 << 33),     # a 2^33-tick gap inside a group: t32 does not fit (build gathers t by index)
    (997, 1 << 40),   # both, plus odd spacing
    (300, 0),         # a group spans 2^24..2^27 ticks: keys carry the event index, t in t32
    (1, 1 << 25),     # 4-byte-key groups before the jump, an index-key group across it
    (97, 0),          # coarse ticks, every group below 2^24: 4-byte keys throughout
])
def test_fast_detect_wide_time_ranges(ecc, orc, gpu, scale, jump):
    W, H = 346, 260
    n = 16384 * 40 + 77  # two groups + a ragged tail
    xy, t, _ = ecc.gen_events(n, seed=41, width=W, height=H)
    t = t.astype(np.int64) * scale
    t[n // 3:] += jump
    o_flags, o_sae = orc.fast_detect(xy, t, W, H)
    g_flags, g_sae = _fast_gpu(ecc, gpu, xy, t, W, H)
    assert o_flags.sum() > 0
    assert (g_flags == o_flags).all(), f"{(g_flags != o_flags).sum()} corner labels differ"
    assert (g_sae == o_sae).all()


@pytest.mark.parametrize("n,wh,mode,seed,slice_events", [
    (600_000, (346, 260), 0, 1, 16384),
    (600_000, (346, 260), 1, 2, 16384),
    (700_000, (1280, 720), 0, 3, 16384),
    (300_000, (640, 480), 1, 4, 16384),
    (100_000, (346, 260), 0, 5, 1000),   # many slices per group, ragged tail
    (400_000, (1600, 900), 1, 6, 16384), # 7475 tiles: flags read the result words without LDS staging
])
def test_fast_detect_matches_oracle(ecc, orc, gpu, n, wh, mode, seed, slice_events):
    W, H = wh
    xy, t, _ = ecc.gen_events(n, seed=seed, width=W, height=H)
    o_flags, o_sae = orc.fast_detect(xy, t, W, H, slice_events=slice_events, border_mode=mode)
    g_flags, g_sae = _fast_gpu(ecc, gpu, xy, t, W, H, border_mode=mode, slice_events=slice_events)
    assert o_flags.sum() > 0, "synthetic stream should contain corners"
    assert (g_flags == o_flags).all(), f"{(g_flags != o_flags).sum()} corner labels differ"
    assert (g_sae == o_sae).all()


def test_fast_detect_stream_continuation(ecc, orc, gpu):
    """Two batches with the SAE carried over == one batch (stream hand-off / sharding)."""
    W, H = W_SMALL, H_SMALL
    xy, t, _ = ecc.gen_events(32768 * 9, seed=8)
    o_flags, o_sae = orc.fast_detect(xy, t, W, H)
    cut = 32768 * 5
    f1, s1 = _fast_gpu(ecc, gpu, xy[:cut], t[:cut], W, H)
    f2, s2 = _fast_gpu(ecc, gpu, xy[cut:], t[cut:], W, H, first_detect=0, sae0=s1)
    assert (np.concatenate([f1, f2]) == o_flags).all()
    assert (s2 == o_sae).all()


@pytest.mark.parametrize("side,groups", [(30, 1.5), (200, 16)])
def test_fast_detect_dense_overflow_path(ecc, orc, gpu, side, groups):
    """Whole slices landing in a side x side patch: every window of the patch holds more values
    than the compact per-pixel lists take, so those items run on the dense-plane kernel (asserted
    through ecc_fast_detect_stats): a few dozen items (30 px) and thousands (200 px, 16 groups).
    Flags and SAE bit-exact."""
    W, H = 346, 260
    rng = np.random.default_rng(5)
    n_dense = int(16384 * 32 * groups)
    xd = rng.integers(150, 150 + side, n_dense)
    yd = rng.integers(100, 100 + side, n_dense)
    td = np.cumsum(rng.integers(0, 3, n_dense)).astype(np.int64)
    xy2, t2, _ = ecc.gen_events(16384 * 50 + 333, seed=17, width=W, height=H)
    xy = np.concatenate([ecc.pack_xy(xd, yd), xy2])
    t = np.concatenate([td, t2 + td[-1] + 1])
    o_flags, o_sae = orc.fast_detect(xy, t, W, H)
    g_flags, g_sae = _fast_gpu(ecc, gpu, xy, t, W, H)
    st = gpu.fast_detect_stats()
    assert st["groups"] >= 3 and st["overflow_items"] > 0, st
    assert (st["overflow_items"] > 1000) == (side == 200), st
    assert o_flags[:n_dense].sum() > 0 and o_flags[n_dense:].sum() > 0
    assert (g_flags == o_flags).all(), f"{(g_flags != o_flags).sum()} corner labels differ"
    assert (g_sae == o_sae).all()


def test_fast_detect_rejects_decreasing_time(ecc, gpu):
    xy, t, _ = ecc.gen_events(40000, seed=2)
    t = t.copy()
    t[20000] = t[19999] - 5
    cfg = ecc.corner_cfg(width=W_SMALL, height=H_SMALL)
    sae = ecc.DeviceArray.zeros(W_SMALL * H_SMALL, np.int64)
    flags = ecc.DeviceArray(len(xy), np.uint8)
    gpu.fast_detect(dev(ecc, xy), dev(ecc, t), len(xy), cfg, sae, flags)
    assert gpu.fast_detect_status() == ecc.ERR_UNSORTED_TIME
    # the error word carries the failing call's tag (no per-call reset): a later sorted call, and
    # a later empty call, report OK; the fused detect + NMS call reports a new failure again
    t_ok = np.sort(t)
    gpu.fast_detect(dev(ecc, xy), dev(ecc, t_ok), len(xy), cfg, sae, flags)
    assert gpu.fast_detect_status() == 0
    gpu.fast_detect(dev(ecc, xy), dev(ecc, t), 0, cfg, sae, flags)
    assert gpu.fast_detect_status() == 0
    ns = -(-len(xy) // cfg.slice_events)
    out, cnt = ecc.DeviceArray(ns * 64, ecc.CORNER_DTYPE), ecc.DeviceArray(ns, np.int32)
    gpu.fast_detect_nms(dev(ecc, xy), dev(ecc, t), len(xy), cfg, sae, flags, 15, 64, out, cnt)
    assert gpu.fast_detect_status() == ecc.ERR_UNSORTED_TIME
    # unsorted -> empty call -> OK (the empty call launches nothing and still reports its own verdict)
    gpu.fast_detect(dev(ecc, xy), dev(ecc, t), 0, cfg, sae, flags)
    assert gpu.fast_detect_status() == 0


def test_fast_detect_status_prepare_finish_verdicts(ecc, gpu):
    """ecc_fast_detect_status over the two-call form (ecc.h): a prepare reports its own batch, a
    finish the batch of its prepare, and an abandoned unsorted prepare leaks into no later call."""
    xy, t, _ = ecc.gen_events(40000, seed=3)
    bad = t.copy()
    bad[30000] = bad[29999] - 7
    cfg = ecc.corner_cfg(width=W_SMALL, height=H_SMALL, first_detect_slice=0)
    n = len(xy)
    d_xy, d_ok, d_bad = dev(ecc, xy), dev(ecc, t), dev(ecc, bad)
    local = ecc.DeviceArray(W_SMALL * H_SMALL, np.int64)
    sae = ecc.DeviceArray.zeros(W_SMALL * H_SMALL, np.int64)
    flags = ecc.DeviceArray(n, np.uint8)
    lib, C = ecc.lib, ecc.C

    def prepare(tt, nn=n):
        ecc.check(lib.ecc_fast_detect_prepare(gpu.ctx, d_xy.ptr, tt.ptr, nn, C.byref(cfg), local.ptr, gpu.stream))

    def finish(tt, nn=n):
        ecc.check(lib.ecc_fast_detect_finish(gpu.ctx, d_xy.ptr, tt.ptr, nn, C.byref(cfg), sae.ptr, flags.ptr,
                                             gpu.stream))

    # unsorted prepare -> its verdict at once; then abandoned, a sorted full call reports OK
    prepare(d_bad)
    assert gpu.fast_detect_status() == ecc.ERR_UNSORTED_TIME
    gpu.fast_detect(d_xy, d_ok, n, cfg, sae, flags)
    assert gpu.fast_detect_status() == 0
    # unsorted prepare (abandoned) -> sorted prepare + finish: OK at both steps
    prepare(d_bad)
    prepare(d_ok)
    assert gpu.fast_detect_status() == 0
    finish(d_ok)
    assert gpu.fast_detect_status() == 0
    # unsorted prepare + finish: the finish reports its prepare's batch
    prepare(d_bad)
    finish(d_bad)
    assert gpu.fast_detect_status() == ecc.ERR_UNSORTED_TIME
    # sorted prepare after it, then an empty prepare: OK
    prepare(d_ok)
    assert gpu.fast_detect_status() == 0
    prepare(d_bad)
    prepare(d_ok, 0)
    assert gpu.fast_detect_status() == 0
    # unsorted prepare, then a sorted fused detect + NMS: OK
    prepare(d_bad)
    ns = -(-n // cfg.slice_events)
    out, cnt = ecc.DeviceArray(ns * 64, ecc.CORNER_DTYPE), ecc.DeviceArray(ns, np.int32)
    gpu.fast_detect_nms(d_xy, d_ok, n, cfg, sae, flags, 15, 64, out, cnt)
    assert gpu.fast_detect_status() == 0


def _any_order_times(kind, n, seed):
    """Timestamps that are NOT non-decreasing: the oracle (the reference's loop) keeps the last
    writer in stream order at every pixel, whatever the times are."""
    rng = np.random.default_rng(seed)
    t = np.cumsum(rng.integers(0, 40, n)).astype(np.int64)
    if kind == "jitter":      # a sensor's slightly out-of-order packets
        t = t + rng.integers(-300, 300, n)
    elif kind == "shuffled":  # every slice's times permuted (ties and reversals everywhere)
        for lo in range(0, n, 16384):
            seg = t[lo:lo + 16384]
            t[lo:lo + 16384] = rng.permutation(seg)
    elif kind == "reversed":  # decreasing stream, negative times, 2^40-tick steps between slices
        t = -(t + (np.arange(n) // 16384).astype(np.int64) * (1 << 40))
    elif kind == "coarse":    # few distinct values: equal times at many circle pixels
        t = rng.integers(0, 8, n).astype(np.int64)
    return t


@pytest.mark.parametrize("kind,mode", [("sorted", 0), ("jitter", 0), ("shuffled", 1), ("reversed", 0),
                                       ("coarse", 0)])
def test_fast_detect_any_order_matches_oracle(ecc, orc, gpu, kind, mode):
    """cfg.any_order = 1: timestamps in any order (Q14's last writer in stream order), every
    group on the exact index-valued path; flags and the final SAE equal the oracle's."""
    W, H = 346, 260
    n = 16384 * 70 + 123  # three groups + a ragged tail
    xy, t0, _ = ecc.gen_events(n, seed=43, width=W, height=H)
    t = t0.astype(np.int64) if kind == "sorted" else _any_order_times(kind, n, 7)
    o_flags, o_sae = orc.fast_detect(xy, t, W, H, border_mode=mode)
    cfg = ecc.corner_cfg(width=W, height=H, border_mode=mode, any_order=1)
    sae = ecc.DeviceArray.zeros(W * H, np.int64)
    flags = ecc.DeviceArray(n, np.uint8)
    gpu.fast_detect(dev(ecc, xy), dev(ecc, t), n, cfg, sae, flags)
    assert gpu.fast_detect_status() == 0
    g_flags = flags.numpy()
    assert o_flags.sum() > 0
    assert (g_flags == o_flags).all(), f"{(g_flags != o_flags).sum()} corner labels differ"
    assert (sae.numpy() == o_sae).all()


def test_fast_detect_any_order_single_call_only(ecc, gpu):
    """The multi-GPU hand-off combines shard images by max time, so any_order is refused there."""
    xy, t, _ = ecc.gen_events(40000, seed=2)
    cfg = ecc.corner_cfg(width=W_SMALL, height=H_SMALL, any_order=1)
    local = ecc.DeviceArray(W_SMALL * H_SMALL, np.int64)
    rc = ecc.lib.ecc_fast_detect_prepare(gpu.ctx, dev(ecc, xy).ptr, dev(ecc, t).ptr, len(xy), ecc.C.byref(cfg),
                                         local.ptr, gpu.stream)
    assert rc == ecc.ERR_INVALID
    cfg.any_order = 2
    sae = ecc.DeviceArray.zeros(W_SMALL * H_SMALL, np.int64)
    flags = ecc.DeviceArray(len(xy), np.uint8)
    with pytest.raises(ecc.EccError):
        gpu.fast_detect(dev(ecc, xy), dev(ecc, t), len(xy), cfg, sae, flags)


def test_arc_test_known_patterns(ecc, orc, gpu):
    """Hand-built SAE patterns around one event (checked by the literal reference loop in the
    oracle): a contiguous fresh arc on both circles is a corner; gaps / ties / too long are not."""
    W, H = 64, 64
    c3 = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    c4 = [(0, 4), (1, 4), (2, 3), (3, 2), (4, 1), (4, 0), (4, -1), (3, -2), (2, -3), (1, -4), (0, -4), (-1, -4), (-2, -3), (-3, -2), (-4, -1), (-4, 0), (-4, 1), (-3, 2), (-2, 3), (-1, 4)]
    cx, cy = 20, 20
    cases = []
    for arc3, arc4, expect in [(range(0, 4), range(0, 5), 1), (range(2, 8), range(3, 11), 1),
                               ([0, 1, 3, 4], range(0, 5), 0), (range(0, 7), range(0, 5), 0),
                               (range(0, 2), range(0, 5), 0), (range(14, 18), range(18, 23), 1),
                               (range(0, 4), range(0, 9), 0)]:
        cases.append((arc3, arc4, expect))
    xs, ts = [], []
    tbase = 1000
    for ci, (arc3, arc4, expect) in enumerate(cases):
        sae = np.zeros((H, W), np.int64)
        for k in arc3:
            dy, dx = c3[k % 16]
            sae[cy + dy, cx + dx] = 500
        for k in arc4:
            dy, dx = c4[k % 20]
            sae[cy + dy, cx + dx] = 500
        assert orc.arc_test(sae.ravel(), W, cx, cy) == expect, ci
    # same patterns through the GPU pipeline: slice 0 paints the pattern, slice 1 holds the event
    for ci, (arc3, arc4, expect) in enumerate(cases):
        pts = set()
        for k in arc3:
            dy, dx = c3[k % 16]
            pts.add((cx + dx, cy + dy))
        for k in arc4:
            dy, dx = c4[k % 20]
            pts.add((cx + dx, cy + dy))
        pts = sorted(pts)
        S = 64
        ev_xy = [ecc.pack_xy(x, y) for x, y in pts] + [ecc.pack_xy(60, 60)] * (S - len(pts))
        ev_t = [500] * S
        ev_xy += [ecc.pack_xy(cx, cy)] + [ecc.pack_xy(2, 2)] * (S - 1)
        ev_t += [600] * S
        xy = np.array(ev_xy, np.uint32)
        t = np.array(ev_t, np.int64)
        o_flags, _ = orc.fast_detect(xy, t, W, H, slice_events=S)
        g_flags, _ = _fast_gpu(ecc, gpu, xy, t, W, H, slice_events=S)
        assert (g_flags == o_flags).all()
        # the centre event itself sees its own pixel as the newest value, not on either circle
        assert g_flags[S] == expect, ci


# ------------------------------------------------------------------------------ NMS
def test_nms_matches_oracle(ecc, orc, gpu):
    W, H = W_SMALL, H_SMALL
    xy, t, _ = ecc.gen_events(1_000_000, seed=21)
    o_flags, _ = orc.fast_detect(xy, t, W, H)
    o_out, o_cnt, rc = orc.corner_nms(xy, o_flags, W, H)
    assert rc == 0 and o_cnt.sum() > 0
    ns = len(o_cnt)
    cap = 4096
    d_out = ecc.DeviceArray(ns * cap, ecc.CORNER_DTYPE)
    d_cnt = ecc.DeviceArray(ns, np.int32)
    gpu.corner_nms(dev(ecc, xy), dev(ecc, o_flags), len(xy), 16384, W, H, 15, cap, d_out, d_cnt)
    gpu.sync()
    g_cnt = d_cnt.numpy()
    assert (g_cnt == o_cnt).all()
    g_out = d_out.numpy()
    for s in range(ns):
        k = o_cnt[s]
        assert (g_out[s * cap: s * cap + k] == o_out[s * cap: s * cap + k]).all(), s


@pytest.mark.parametrize("W,H,n,S,box,cap", [
    (346, 260, 16384 * 40 + 333, 16384, 15, 4096),  # fused candidates, ragged last slice (333 % 4 = 1)
    (346, 260, 4096 * 30 + 2, 4096, 15, 40),        # short slices, capacity hit
    (240, 180, 12288 * 9, 12288, 8, 4096),          # even box
    (346, 260, 6000 * 12, 6000, 15, 4096),          # S % 4 == 0 but not a power of two
    (346, 260, 1001 * 40, 1001, 15, 4096),          # S % 4 != 0: the two-call path
    (346, 260, 16384 * 8, 16384, 1, 4096),          # 1-px cells: the kept-list NMS kernel
])
def test_fast_detect_nms_matches_two_calls_and_oracle(ecc, orc, gpu, W, H, n, S, box, cap):
    """ecc_fast_detect_nms (the flag pass writes the NMS candidate lists) == ecc_fast_detect +
    ecc_corner_nms == the oracle: flags, final SAE, per-slice kept corners and the status."""
    xy, t, _ = ecc.gen_events(n, seed=n % 1000 + box, width=W, height=H)
    o_flags, o_sae = orc.fast_detect(xy, t, W, H, slice_events=S)
    o_out, o_cnt, rc = orc.corner_nms(xy, o_flags, W, H, box=box, cap=cap, slice_events=S)
    ns = len(o_cnt)
    cfg = ecc.corner_cfg(width=W, height=H, slice_events=S)
    sae = dev(ecc, np.zeros(W * H, np.int64))
    flags = ecc.DeviceArray(n, np.uint8)
    d_out = ecc.DeviceArray(ns * cap, ecc.CORNER_DTYPE)
    d_cnt = ecc.DeviceArray(ns, np.int32)
    gpu.fast_detect_nms(dev(ecc, xy), dev(ecc, t), n, cfg, sae, flags, box, cap, d_out, d_cnt)
    assert gpu.fast_detect_status() == 0
    assert gpu.corner_nms_status() == (ecc.ERR_CAPACITY if rc else 0)
    assert (flags.numpy() == o_flags).all()
    assert (sae.numpy() == o_sae).all()
    assert (d_cnt.numpy() == o_cnt).all()
    g_out = d_out.numpy()
    for s in range(ns):
        k = o_cnt[s]
        assert (g_out[s * cap: s * cap + k] == o_out[s * cap: s * cap + k]).all(), s


def test_nms_dense_candidates(ecc, orc, gpu):
    """Many overlapping candidates in one slice (within-chunk dependency resolution)."""
    W, H = 200, 200
    rng = np.random.default_rng(4)
    n = 16384
    x = rng.integers(4, 196, n)
    y = rng.integers(4, 196, n)
    xy = ecc.pack_xy(x, y)
    flags = (rng.random(n) < 0.7).astype(np.uint8)
    o_out, o_cnt, _ = orc.corner_nms(xy, flags, W, H, slice_events=n)
    d_out = ecc.DeviceArray(4096, ecc.CORNER_DTYPE)
    d_cnt = ecc.DeviceArray(1, np.int32)
    gpu.corner_nms(dev(ecc, xy), dev(ecc, flags), n, n, W, H, 15, 4096, d_out, d_cnt)
    gpu.sync()
    k = o_cnt[0]
    assert d_cnt.numpy()[0] == k
    assert (d_out.numpy()[:k] == o_out[:k]).all()
    assert gpu.corner_nms_status() == 0


@pytest.mark.parametrize("box,wh,density", [
    (15, (346, 260), 0.05),   # grid kernel, reference box
    (8, (346, 260), 0.3),     # even box size (half = 4)
    (31, (640, 480), 0.5),    # large boxes
    (1, (346, 260), 0.2),     # 1-pixel cells: grid too large for LDS -> kept-list kernel
    (15, (1280, 720), 0.02),  # reference sensor
])
def test_nms_box_sizes(ecc, orc, gpu, box, wh, density):
    W, H = wh
    rng = np.random.default_rng(box * 7 + W)
    n = 16384 * 5 + 333  # ragged last slice
    xy = ecc.pack_xy(rng.integers(0, W, n), rng.integers(0, H, n))
    flags = (rng.random(n) < density).astype(np.uint8)
    cap = 8192
    o_out, o_cnt, rc = orc.corner_nms(xy, flags, W, H, box=box, cap=cap)
    assert rc == 0
    ns = len(o_cnt)
    d_out = ecc.DeviceArray(ns * cap, ecc.CORNER_DTYPE)
    d_cnt = ecc.DeviceArray(ns, np.int32)
    gpu.corner_nms(dev(ecc, xy), dev(ecc, flags), n, 16384, W, H, box, cap, d_out, d_cnt)
    assert gpu.corner_nms_status() == 0
    assert (d_cnt.numpy() == o_cnt).all()
    g_out = d_out.numpy()
    for s in range(ns):
        k = o_cnt[s]
        assert (g_out[s * cap: s * cap + k] == o_out[s * cap: s * cap + k]).all(), s


@pytest.mark.parametrize("cap", [8192, 40])
def test_nms_parallel_and_greedy_slices(ecc, orc, gpu, cap):
    """Slices below and above the parallel pass's 2048-candidate limit in one call, including
    long dependency chains (a diagonal staircase: every candidate overlaps its predecessor),
    a slice with exactly 2048 candidates and one with 2049, and an empty slice."""
    W, H = 346, 260
    rng = np.random.default_rng(77)
    S = 4096
    xs, ys, fl = [], [], []
    for k, m in enumerate([300, 2048, 2049, 0, 3000, 1000, 2047]):
        if k == 5:  # staircase in event order, then random order of a second one
            t = np.arange(m)
            x, y = (t * 3) % 340, (t // 113) * 9 % 250
        elif k == 6:
            t = rng.permutation(m)
            x, y = (t % 300), (t // 300) * 2
        else:
            x, y = rng.integers(0, W, S), rng.integers(0, H, S)
        f = np.zeros(S, np.uint8)
        if k in (5, 6):
            x = np.concatenate([x, rng.integers(0, W, S - m)])
            y = np.concatenate([y, rng.integers(0, H, S - m)])
            f[:m] = 1
        else:
            f[rng.choice(S, m, replace=False)] = 1
        xs.append(x), ys.append(y), fl.append(f)
    xy = ecc.pack_xy(np.concatenate(xs), np.concatenate(ys))
    flags = np.concatenate(fl)
    n = len(xy)
    o_out, o_cnt, rc = orc.corner_nms(xy, flags, W, H, cap=cap, slice_events=S)
    ns = len(o_cnt)
    d_out = ecc.DeviceArray(ns * cap, ecc.CORNER_DTYPE)
    d_cnt = ecc.DeviceArray(ns, np.int32)
    gpu.corner_nms(dev(ecc, xy), dev(ecc, flags), n, S, W, H, 15, cap, d_out, d_cnt)
    assert gpu.corner_nms_status() == (ecc.ERR_CAPACITY if rc else 0)
    assert (d_cnt.numpy() == o_cnt).all()
    g_out = d_out.numpy()
    for s in range(ns):
        k = o_cnt[s]
        assert (g_out[s * cap: s * cap + k] == o_out[s * cap: s * cap + k]).all(), s


def test_nms_status_capacity_and_outside(ecc, gpu):
    W, H = 346, 260
    rng = np.random.default_rng(9)
    n = 16384
    xy = ecc.pack_xy(rng.integers(0, W, n), rng.integers(0, H, n))
    flags = np.ones(n, np.uint8)
    d_out = ecc.DeviceArray(8, ecc.CORNER_DTYPE)
    d_cnt = ecc.DeviceArray(1, np.int32)
    gpu.corner_nms(dev(ecc, xy), dev(ecc, flags), n, n, W, H, 15, 8, d_out, d_cnt)
    assert gpu.corner_nms_status() == ecc.ERR_CAPACITY
    assert d_cnt.numpy()[0] == 8
    xy2 = xy.copy()
    xy2[5] = ecc.pack_xy(np.array([W + 3]), np.array([10]))[0]  # flagged event outside the image
    d_out = ecc.DeviceArray(4096, ecc.CORNER_DTYPE)
    gpu.corner_nms(dev(ecc, xy2), dev(ecc, flags), n, n, W, H, 15, 4096, d_out, d_cnt)
    assert gpu.corner_nms_status() == ecc.ERR_INVALID
    sparse = np.zeros(n, np.uint8)  # the same on the parallel pass (few candidates)
    sparse[::64] = 1
    sparse[5] = 1
    gpu.corner_nms(dev(ecc, xy2), dev(ecc, sparse), n, n, W, H, 15, 4096, d_out, d_cnt)
    assert gpu.corner_nms_status() == ecc.ERR_INVALID


# ------------------------------------------------------------------------------ tracker
def _track_key(tr):
    return (tr.x, tr.y, tr.label, tr.frame_count, tr.is_matched, tr.frames_since_last_detection,
            tr.hist_len, tuple(tr.hist_x[:tr.hist_len]), tuple(tr.hist_y[:tr.hist_len]),
            np.float32(tr.vx).view(np.uint32), np.float32(tr.vy).view(np.uint32),
            np.float32(tr.dir_cur_x).view(np.uint32), np.float32(tr.dir_cur_y).view(np.uint32),
            tr.group_id)


def test_tracker_matches_oracle(ecc, orc, gpu):
    W, H = W_SMALL, H_SMALL
    xy, t, _ = ecc.gen_events(16384 * 48, seed=31)
    o_flags, _ = orc.fast_detect(xy, t, W, H)
    cap = 4096
    o_out, o_cnt, _ = orc.corner_nms(xy, o_flags, W, H, cap=cap)
    ns = len(o_cnt)
    otr = orc.OracleTracker(ecc.tracker_cfg())
    gtr = ecc.Tracker(gpu)
    d_out, d_cnt = dev(ecc, o_out), dev(ecc, o_cnt)
    # feed in two device launches (16 + rest slices) to exercise state carry-over
    for s in range(ns):
        otr.update(o_out[s * cap: s * cap + o_cnt[s]])
    sub = 16
    gtr.update(d_out, d_cnt, sub, cap)
    rest_out = dev(ecc, o_out[sub * cap:])
    rest_cnt = dev(ecc, o_cnt[sub:])
    gtr.update(rest_out, rest_cnt, ns - sub, cap)
    gpu.sync()
    assert gtr.status() == 0
    o_tr = otr.tracks(ecc.Track)
    g_tr = gtr.tracks()
    assert len(o_tr) > 0 and len(g_tr) == len(o_tr)
    for a, b in zip(g_tr, o_tr):
        assert _track_key(a) == _track_key(b)
    og, ol = otr.groups(ecc.Group)
    gg, gl = gtr.groups()
    assert len(gg) == len(og)
    for a, b in zip(gg, og):
        assert (a.id, a.n_labels, a.first_label_offset) == (b.id, b.n_labels, b.first_label_offset)
        for f in ("avg_vx", "avg_vy", "cx", "cy", "radius"):
            assert np.float32(getattr(a, f)) == np.float32(getattr(b, f)), f
    nl = sum(g.n_labels for g in og)
    assert (gl[:nl] == ol[:nl]).all()


def _compare_trackers(ecc, gtr, otr):
    o_tr = otr.tracks(ecc.Track)
    g_tr = gtr.tracks()
    assert len(g_tr) == len(o_tr)
    for a, b in zip(g_tr, o_tr):
        assert _track_key(a) == _track_key(b)
    og, ol = otr.groups(ecc.Group)
    gg, gl = gtr.groups()
    assert len(gg) == len(og)
    for a, b in zip(gg, og):
        assert (a.id, a.n_labels, a.first_label_offset) == (b.id, b.n_labels, b.first_label_offset)
        for f in ("avg_vx", "avg_vy", "cx", "cy", "radius"):
            assert np.float32(getattr(a, f)) == np.float32(getattr(b, f)), f
    nl = sum(g.n_labels for g in og)
    assert (gl[:nl] == ol[:nl]).all()
    return len(o_tr), len(og)


def _dense_detections(seed, n_slices, per_slice, n_centres, spread, W=346, H=260):
    """Clustered detections drifting slowly: many tracks compete for the same detections, so
    the matching takes several conflict rounds (order-dependent greedy claims)."""
    rng = np.random.default_rng(seed)
    c = rng.uniform([20, 20], [W - 20, H - 20], size=(n_centres, 2))
    v = rng.uniform(-3, 3, size=(n_centres, 2))
    out = []
    for s in range(n_slices):
        n = int(rng.integers(per_slice // 2, per_slice + 1))
        k = rng.integers(0, n_centres, size=n)
        pts = np.rint(c[k] + rng.normal(0, spread, size=(n, 2))).astype(np.int32)
        arr = np.zeros(n, np.dtype([("x", np.int32), ("y", np.int32), ("label", np.int32)]))
        arr["x"], arr["y"] = pts[:, 0], pts[:, 1]
        out.append(arr)
        c += v
    return out


@pytest.mark.parametrize("seed,per_slice,n_centres,spread,cfg_over", [
    (51, 120, 12, 8.0, {}),
    (52, 400, 30, 12.0, {}),
    (53, 60, 4, 20.0, {"max_frames": 3, "frames_to_skip": 1, "history_size": 16, "group_radius": 40.0}),
    (54, 900, 80, 6.0, {"max_distance": 12.5, "damping": 0.5, "smoothing": 0.6}),
    (56, 500, 40, 10.0, {"max_distance": 1.0e6}),                   # radius too large for the grid
    (57, 450, 30, 15.0, {"max_distance": 45.0, "group_radius": -1.0}),  # no group ever forms
    # short-lived tracks keep T + C <= 256 (tracker_fast_kernel) while every track has far more
    # than 8 detections in range (its list overflows: the rounds rescan) ...
    (58, 120, 2, 4.0, {"max_frames": 2, "frames_to_skip": 1}),
    # ... or more than 64 tracks stay unresolved after round 0 (workgroup-wide rounds), C > 64
    (59, 110, 40, 2.0, {"max_frames": 2, "frames_to_skip": 1, "max_distance": 12.0}),
    # C > 128 with few tracks: a track's merged candidate list is not in detection order, and
    # integer detections around a prediction tie in distance (first minimum = smallest index)
    (60, 200, 3, 6.0, {"max_frames": 2, "frames_to_skip": 1}),
    (61, 220, 2, 3.0, {"max_frames": 1, "frames_to_skip": 1, "max_distance": 8.0}),
])
def test_tracker_dense_conflicts_match_oracle(ecc, orc, gpu, seed, per_slice, n_centres, spread, cfg_over):
    cfg = ecc.tracker_cfg(**cfg_over)
    dets = _dense_detections(seed, 36, per_slice, n_centres, spread)
    cap = max(len(d) for d in dets)
    ns = len(dets)
    flat = np.zeros(ns * cap, ecc.CORNER_DTYPE)
    cnt = np.zeros(ns, np.int32)
    for s, d in enumerate(dets):
        flat[s * cap: s * cap + len(d)] = d
        cnt[s] = len(d)
    otr = orc.OracleTracker(cfg)
    for d in dets:
        otr.update(d)
    gtr = ecc.Tracker(gpu, cfg)
    # three launches (1, 20, rest slices): state carries across launches
    bounds = [0, 1, 21, ns]
    for a, b in zip(bounds[:-1], bounds[1:]):
        gtr.update(dev(ecc, flat[a * cap: b * cap]), dev(ecc, cnt[a:b]), b - a, cap)
    gpu.sync()
    assert gtr.status() == 0
    n_tr, n_gr = _compare_trackers(ecc, gtr, otr)
    assert n_tr > 0 and (n_gr > 0) == (cfg.group_radius >= 0)


def test_corner_pack_and_tracker_lists_match_strided(ecc, orc, gpu):
    """ecc_corner_pack == the per-slice lists packed on the host, and the tracker over explicit
    lists (two 'shards' packed separately, at distinct bases with a gap, as the multi-GPU merge
    gathers them) == the tracker over the cap-strided NMS output == the oracle."""
    W, H = 346, 260
    n = 16384 * 36
    xy, t, _ = ecc.gen_events(n, seed=23, width=W, height=H)
    o_flags, _ = orc.fast_detect(xy, t, W, H)
    ns, cap = n // 16384, 4096
    o_out, o_cnt, _ = orc.corner_nms(xy, o_flags, W, H, cap=cap)
    d_out, d_cnt = dev(ecc, o_out), dev(ecc, o_cnt)
    half = ns // 2
    packed = ecc.DeviceArray(ns * cap + 1000, ecc.CORNER_DTYPE)
    offs = ecc.DeviceArray(ns + 2, np.int64)
    # shard A: slices [0, half) at element 0; shard B: slices [half, ns) at element base_b
    base_b = int(o_cnt[:half].sum()) + 1000
    gpu.corner_pack(d_out, d_cnt, half, cap, packed, offs)
    ecc.check(ecc.lib.ecc_corner_pack(gpu.ctx, d_out.ptr + half * cap * 12, d_cnt.ptr + half * 4, ns - half, cap,
                                      packed.ptr + base_b * 12, offs.ptr + (half + 1) * 8, gpu.stream))
    gpu.sync()
    off = offs.numpy()
    assert off[half] == o_cnt[:half].sum() and off[ns + 1] == o_cnt[half:].sum()
    starts = np.concatenate([off[:half], base_b + off[half + 1: ns + 1]]).astype(np.int64)
    host_pk = packed.numpy()
    for s in range(ns):
        assert np.array_equal(host_pk[starts[s]: starts[s] + o_cnt[s]], o_out[s * cap: s * cap + o_cnt[s]])
    g1 = ecc.Tracker(gpu)
    g1.update(d_out, d_cnt, ns, cap)
    g2 = ecc.Tracker(gpu)
    g2.update_lists(packed, dev(ecc, starts), d_cnt, ns)
    otr = orc.OracleTracker(ecc.tracker_cfg())
    for s in range(ns):
        otr.update(o_out[s * cap: s * cap + o_cnt[s]])
    ref = [_track_key(tr) for tr in otr.tracks(ecc.Track)]
    assert len(ref) > 0
    assert [_track_key(tr) for tr in g1.tracks()] == ref
    assert [_track_key(tr) for tr in g2.tracks()] == ref
    assert g1.status() == 0 and g2.status() == 0


def test_tracker_fast_path_handover_matches_oracle(ecc, orc, gpu):
    """tracker_fast_kernel (T + C <= 256 per slice, state in registers) hands a launch over to
    tracker_kernel at the first slice above that bound; the next launch starts on the fast path
    again once the list is small.  Sparse -> dense -> sparse slices, three launches, vs the oracle."""
    sparse = _dense_detections(61, 30, 40, 6, 10.0)
    dense = _dense_detections(62, 6, 700, 60, 8.0)
    dets = sparse[:12] + dense + sparse[12:]
    cfg = ecc.tracker_cfg(max_frames=4, frames_to_skip=2)  # short-lived tracks: T falls again
    cap = max(len(d) for d in dets)
    ns = len(dets)
    flat = np.zeros(ns * cap, ecc.CORNER_DTYPE)
    cnt = np.zeros(ns, np.int32)
    for s, d in enumerate(dets):
        flat[s * cap: s * cap + len(d)] = d
        cnt[s] = len(d)
    otr = orc.OracleTracker(cfg)
    gtr = ecc.Tracker(gpu, cfg)
    bounds = [0, 15, 26, ns]  # launch 1 hands over at slice 12; launch 2 starts above 256
    for a, b in zip(bounds[:-1], bounds[1:]):
        for d in dets[a:b]:
            otr.update(d)
        gtr.update(dev(ecc, flat[a * cap: b * cap]), dev(ecc, cnt[a:b]), b - a, cap)
        gpu.sync()
        assert gtr.status() == 0
        n_tr, _ = _compare_trackers(ecc, gtr, otr)
        assert n_tr > 0


@pytest.mark.parametrize("per_slice,max_tracks", [(300, 64), (40, 16)])  # general / fast kernel
def test_tracker_capacity_flag(ecc, gpu, per_slice, max_tracks):
    """More new tracks than max_tracks: the overflow is dropped and reported."""
    dets = _dense_detections(55, 4, per_slice, 40, 30.0)
    cap = max(len(d) for d in dets)
    flat = np.zeros(4 * cap, ecc.CORNER_DTYPE)
    cnt = np.zeros(4, np.int32)
    for s, d in enumerate(dets):
        flat[s * cap: s * cap + len(d)] = d
        cnt[s] = len(d)
    gtr = ecc.Tracker(gpu, max_tracks=max_tracks)
    gtr.update(dev(ecc, flat), dev(ecc, cnt), 4, cap)
    gpu.sync()
    assert gtr.status() == ecc.ERR_CAPACITY
    assert len(gtr.tracks()) <= max_tracks


# ------------------------------------------------------------------------------ eps-neighbourhoods
@pytest.mark.parametrize("eps,min_pts", [(10.0, 2), (20.0, 20), (1.01, 1), (3.5, 64)])
def test_eps_neighbourhoods_match_oracle(ecc, orc, gpu, eps, min_pts):
    xy, _, _ = ecc.gen_events(60_000, seed=41)
    rep_xy, _, u, _ = orc.downsample_hash(xy)
    nw = len(u)
    o_cnt, o_core, o_off, o_nbr = orc.eps_neighbours(rep_xy, nw, 8192, u, eps, min_pts)
    d_xy, d_u = dev(ecc, rep_xy), dev(ecc, u)
    d_cnt = ecc.DeviceArray(nw * 8192, np.int32)
    d_core = ecc.DeviceArray(nw * 8192, np.float64)
    gpu.eps_counts(d_xy, nw, 8192, d_u, eps, min_pts, d_cnt, d_core)
    d_off = ecc.DeviceArray(nw * 8192 + 1, np.int64)
    cap = int(o_off[-1]) + 16
    d_nbr = ecc.DeviceArray(cap, np.int32)
    gpu.eps_lists(d_xy, nw, 8192, d_u, eps, d_cnt, d_off, d_nbr, cap)
    gpu.sync()
    g_cnt, g_core, g_off = d_cnt.numpy(), d_core.numpy(), d_off.numpy()
    for w in range(nw):
        sl = slice(w * 8192, w * 8192 + u[w])
        assert (g_cnt[sl] == o_cnt[sl]).all()
        assert np.array_equal(g_core[sl], o_core[sl])
    assert (g_off == o_off).all()
    assert (d_nbr.numpy()[:o_off[-1]] == o_nbr[:o_off[-1]]).all()


@pytest.mark.parametrize("eps,min_pts", [(6.0, 64), (12.5, 20), (3.0, 3)])
def test_eps_counts_wide_segments(ecc, orc, gpu, eps, min_pts):
    """16384-point segments (dynamic LDS above 64 KiB) and the min_pts-sized core networks; the
    lists of the same segments (bitmap words of 4 per lane, thousands of neighbours per query)."""
    rng = np.random.default_rng(61)
    n_segs, stride = 2, 16384
    counts = np.array([16384, 9001], np.int32)
    n = n_segs * stride
    blob = rng.normal([170, 130], 9.0, size=(n, 2))
    noise = rng.uniform([0, 0], [346, 260], size=(n, 2))
    pick = rng.random(n) < 0.6
    pts = np.clip(np.rint(np.where(pick[:, None], blob, noise)), 0, [345, 259]).astype(np.int64)
    pts[100:140] = pts[99]  # duplicates
    xy = ecc.pack_xy(pts[:, 0], pts[:, 1])
    o_cnt, o_core, o_off, o_nbr = orc.eps_neighbours(xy, n_segs, stride, counts, eps, min_pts)
    d_cnt = ecc.DeviceArray(n, np.int32)
    d_core = ecc.DeviceArray(n, np.float64)
    gpu.eps_counts(dev(ecc, xy), n_segs, stride, dev(ecc, counts), eps, min_pts, d_cnt, d_core)
    d_off = ecc.DeviceArray(n + 1, np.int64)
    d_nbr = ecc.DeviceArray(int(o_off[-1]) + 16, np.int32)
    gpu.eps_lists(dev(ecc, xy), n_segs, stride, dev(ecc, counts), eps, d_cnt, d_off, d_nbr, int(o_off[-1]) + 16)
    gpu.sync()
    import ctypes as C
    total = C.c_int64(0)
    assert ecc.lib.ecc_eps_total(gpu.ctx, d_off.ptr, n, C.byref(total), gpu.stream) == 0  # no list error
    assert (d_off.numpy() == o_off).all() and total.value == o_off[-1]
    assert (d_nbr.numpy()[:o_off[-1]] == o_nbr[:o_off[-1]]).all()
    g_cnt, g_core = d_cnt.numpy(), d_core.numpy()
    for sgi in range(n_segs):
        sl = slice(sgi * stride, sgi * stride + counts[sgi])
        assert (g_cnt[sl] == o_cnt[sl]).all()
        assert np.array_equal(g_core[sl], o_core[sl])
        pad = slice(sgi * stride + counts[sgi], (sgi + 1) * stride)
        assert (g_cnt[pad] == 0).all() and (g_core[pad] == -1.0).all()


@pytest.mark.parametrize("min_pts", [0, 2, 5, 20])
@pytest.mark.parametrize("eps", [0.5, 1.01, 10.0, 20.0, 31.9, 37.9, 400.0])
def test_eps_counts_row_run_matches_oracle(ecc, orc, gpu, eps, min_pts):
    """The row-run bitmap kernel (counts; with min_pts > 0 also core distances) on downsample
    windows (distinct pixels), plus segments it must leave to the candidate walk — a repeated
    pixel, a bounding box above its LDS bitmap — an empty segment and a full 8192-point segment;
    padding counts 0 and core distance -1."""
    xy, _, _ = ecc.gen_events(60_000, seed=43)
    rep_xy, _, u, _ = orc.downsample_hash(xy)
    rng = np.random.default_rng(7)
    stride = 8192
    segs, counts = [], []
    for w in range(len(u)):
        segs.append(rep_xy[w * stride:(w + 1) * stride])
        counts.append(int(u[w]))
    dup = rep_xy[:stride].copy()
    dup[5] = dup[17]  # one repeated pixel
    segs.append(dup); counts.append(int(u[0]))
    wide = ecc.pack_xy(rng.integers(0, 3000, stride), rng.integers(0, 2000, stride))  # 2000 x 94 words
    segs.append(wide); counts.append(3000)
    segs.append(np.zeros(stride, np.uint32)); counts.append(0)
    pix = rng.permutation(346 * 260)[:stride]  # 8192 distinct pixels
    segs.append(ecc.pack_xy(pix % 346, pix // 346)); counts.append(stride)
    allxy = np.concatenate(segs).astype(np.uint32)
    counts = np.array(counts, np.int32)
    n_segs = len(counts)
    o_cnt, o_core, _, _ = orc.eps_neighbours(allxy, n_segs, stride, counts, eps, max(min_pts, 1), want_lists=False)
    d_cnt = ecc.DeviceArray(n_segs * stride, np.int32)
    d_core = ecc.DeviceArray(n_segs * stride, np.float64) if min_pts else None
    gpu.eps_counts(dev(ecc, allxy), n_segs, stride, dev(ecc, counts), eps, max(min_pts, 1), d_cnt, d_core)
    gpu.sync()
    g_cnt = d_cnt.numpy()
    g_core = d_core.numpy() if min_pts else None
    for sgi in range(n_segs):
        sl = slice(sgi * stride, sgi * stride + counts[sgi])
        pad = slice(sgi * stride + counts[sgi], (sgi + 1) * stride)
        assert (g_cnt[sl] == o_cnt[sl]).all(), sgi
        assert (g_cnt[pad] == 0).all(), sgi
        if min_pts:
            assert np.array_equal(g_core[sl], o_core[sl]), sgi
            assert (g_core[pad] == -1.0).all(), sgi


def test_eps_duplicates_and_kdtree_kat(ecc, gpu):
    """kd-tree KATs of OPT/test/test_main.cpp:595-720 (radius 1.01), 1-D cases mapped onto the
    x axis (+4), including the duplicate-point case."""
    import json
    from pathlib import Path
    kat = json.loads((Path(__file__).parent / "golden" / "optics_kat.json").read_text())
    for name, shift in (("kdtree_1d", 4), ("kdtree_1d_dup", 1), ("kdtree_2d", 0)):
        case = kat[name]
        pts = np.array(case["points"], np.float64)
        if pts.shape[1] == 1:
            pts = np.concatenate([pts + shift, np.zeros_like(pts)], 1)
        xy = ecc.pack_xy(pts[:, 0].astype(np.int64), pts[:, 1].astype(np.int64))
        n = len(xy)
        d_cnt = ecc.DeviceArray(n, np.int32)
        gpu.eps_counts(dev(ecc, xy), 1, n, None, case["radius"], 1, d_cnt, None)
        d_off = ecc.DeviceArray(n + 1, np.int64)
        d_nbr = ecc.DeviceArray(n * n, np.int32)
        gpu.eps_lists(dev(ecc, xy), 1, n, None, case["radius"], d_cnt, d_off, d_nbr, n * n)
        gpu.sync()
        off, nbr = d_off.numpy(), d_nbr.numpy()
        for q, expected in case["queries"]:
            q = np.array(q, np.float64)
            if len(q) == 1:
                q = np.array([q[0] + shift, 0.0])
            i = int(np.where((pts == q).all(1))[0][0])
            assert list(nbr[off[i]:off[i + 1]]) == expected, (name, q)


# ------------------------------------------------------------------------------ BASELINE config C3
@pytest.fixture(scope="module")
def c3_points(ecc, orc):
    """C3: k-means k=16 on 50 M points = the representatives of a 10 M-event 346x260 batch (C2)
    tiled to 50 M, as packed u16 and as interleaved float; plus the oracle's 3-pass k-means."""
    xy, _, _ = ecc.gen_events(10_000_000, seed=12, width=346, height=260)
    rx, _, u, _ = orc.downsample_hash(xy)
    dense = np.concatenate([rx[w * 8192: w * 8192 + u[w]] for w in range(len(u))])
    n = 50_000_000
    pts = np.resize(dense, n)
    c0 = np.stack([np.linspace(20, 326, 16), np.linspace(20, 240, 16)[::-1]], 1).astype(np.float32).ravel()
    o_c, o_lab, o_it = orc.kmeans_run_xy16(pts, c0, 3)
    return pts, c0, o_c, o_lab, o_it


@pytest.mark.parametrize("frame", [None, (346, 260), (300, 200)])
def test_kmeans_c3_xy16_50m(ecc, gpu, c3_points, frame):
    """Bounding-box form, the sensor frame, and a frame smaller than the points' extent (the
    points outside it are assigned one by one): all equal the oracle."""
    pts, c0, o_c, o_lab, o_it = c3_points
    n = len(pts)
    d_c, d_lab, d_it = dev(ecc, c0), ecc.DeviceArray(n, np.uint8), ecc.DeviceArray(1, np.int32)
    cfg = ecc.kmeans_cfg(k=16, max_iters=3, tol=-1.0)
    if frame is None:
        gpu.kmeans_xy16(dev(ecc, pts), 1, n, None, d_c, cfg, d_lab, d_it)
    else:
        gpu.kmeans_xy16_frame(dev(ecc, pts), 1, n, None, frame[0], frame[1], d_c, cfg, d_lab, d_it)
    gpu.sync()
    assert d_it.numpy()[0] == o_it
    assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32))
    assert (d_lab.numpy() == o_lab).all()


@pytest.mark.parametrize("wh,frame,k", [
    ((346, 260), (346, 260), 16),  # label image staged in LDS (90 KB)
    ((346, 260), (346, 260), 24),  # the same with the K = 32 kernels
    ((480, 360), (480, 360), 16),  # 173 KB frame: labels gathered from the global image
    ((346, 260), (300, 200), 20),  # points outside the frame: assigned one by one
])
def test_kmeans_frame_segments_match_oracle(ecc, orc, gpu, wh, frame, k):
    """The bench's layout: downsample windows of 8192 slots with per-window counts (ragged last
    window, whose buffer ends at its count), through the frame path's count kernel and both
    label kernels; centroids and every label equal the oracle's over the dense points."""
    W, H = wh
    n = 8192 * 300 + 1111
    xy, _, _ = ecc.gen_events(n, seed=29, width=W, height=H)
    rx, _, u, _ = orc.downsample_hash(xy)
    nw = len(u)
    dense = np.concatenate([rx[w * 8192: w * 8192 + u[w]] for w in range(nw)])
    buf = rx[: (nw - 1) * 8192 + u[-1]].copy()  # no slack after the last window's points
    c0 = np.stack([np.linspace(10, W - 10, k), np.linspace(10, H - 10, k)[::-1]], 1).astype(np.float32).ravel()
    o_c, o_lab, o_it = orc.kmeans_run_xy16(dense, c0, 4)
    d_c, d_lab = dev(ecc, c0), ecc.DeviceArray(nw * 8192, np.uint8)
    cfg = ecc.kmeans_cfg(k=k, max_iters=4, tol=-1.0)
    gpu.kmeans_xy16_frame(dev(ecc, buf), nw, 8192, dev(ecc, u.astype(np.int32)), frame[0], frame[1], d_c, cfg, d_lab)
    gpu.sync()
    assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32))
    g_lab = d_lab.numpy()
    g_dense = np.concatenate([g_lab[w * 8192: w * 8192 + u[w]] for w in range(nw)])
    assert (g_dense == o_lab).all()


@pytest.mark.parametrize("case", ["demo", "ints_full_bins", "floats", "empty_cluster", "one_pass", "few"])
def test_kmeans_refcompat_matches_oracle(ecc, orc, gpu, case):
    """ecc_kmeans_refcompat_f32 (the reference's own loop, Q7-Q9) against orc_kmeans_refcompat,
    whose passes tests/test_ref_opencl.py pins against the reference kernels: the pass count, the
    centroids, the last pass's bin counts and chunk sums, bit for bit.  Cases: the reference's demo
    data and centres (KM/assign_to_centers2.c), 16 384 integer points (bins past 2 048: counted,
    not stored), non-integer floats (the chunk sums' tree order matters), a centre no point reaches
    (0/0 in the update: C's int abs of NaN), one pass, three points."""
    rng = np.random.default_rng(5)
    c0 = np.array([1, 1, 10, 10, 20, 20, 30, 30, 50, 50, 60, 60, 70, 70, 80, 80], np.float32)
    max_passes = 50
    if case == "demo":
        pts = (np.arange(4096) % 100).astype(np.float32)
    elif case == "ints_full_bins":
        pts = rng.integers(0, 100, 2 * 16384).astype(np.float32)
    elif case == "floats":
        pts = (rng.random(2 * 5000) * 90).astype(np.float32)
    elif case == "empty_cluster":
        pts = (rng.random(2 * 3000) * 40).astype(np.float32)
        c0 = c0.copy()
        c0[14:] = 1000.0  # unreachable centre (threshold 50)
    elif case == "one_pass":
        pts = rng.integers(0, 100, 2 * 4000).astype(np.float32)
        max_passes = 1
    else:
        pts = np.array([3, 4, 55, 56, 81, 79], np.float32)
    n = len(pts) // 2
    o_c, o_cnt, o_ss = c0.copy(), np.zeros(8, np.int32), np.zeros(32, np.float32)
    o_p = orc.lib.orc_kmeans_refcompat(pts.ctypes.data, n, o_c.ctypes.data, max_passes, o_cnt.ctypes.data,
                                       o_ss.ctypes.data)
    d_c, d_p, d_cnt, d_ss = dev(ecc, c0), ecc.DeviceArray(1, np.int32), ecc.DeviceArray(8, np.int32), ecc.DeviceArray(32, np.float32)
    ecc.check(ecc.lib.ecc_kmeans_refcompat_f32(gpu.ctx, dev(ecc, pts).ptr, n, d_c.ptr, max_passes, d_p.ptr, d_cnt.ptr,
                                               d_ss.ptr, gpu.stream))
    gpu.sync()
    assert int(d_p.numpy()[0]) == o_p, (d_p.numpy(), o_p)
    assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32)), (d_c.numpy(), o_c)
    assert np.array_equal(d_cnt.numpy(), o_cnt), (d_cnt.numpy(), o_cnt)
    assert np.array_equal(d_ss.numpy().view(np.uint32), o_ss.view(np.uint32)), (d_ss.numpy(), o_ss)
    if case == "ints_full_bins":
        assert o_cnt.max() > 2048  # the case really overflows a bin
    if case == "empty_cluster":
        assert o_cnt[7] == 0
    assert ecc.lib.ecc_kmeans_refcompat_f32(gpu.ctx, None, 16385, d_c.ptr, 5, None, None, None, gpu.stream) == ecc.ERR_INVALID


@pytest.mark.parametrize("engine", [1, 2, 3])
def test_kmeans_c3_f32_50m(ecc, gpu, c3_points, engine):
    pts, c0, o_c, o_lab, o_it = c3_points
    n = len(pts)
    x, y = ecc.unpack_xy(pts)
    f = np.empty(2 * n, np.float32)
    f[0::2], f[1::2] = x, y
    d_c, d_lab, d_it = dev(ecc, c0), ecc.DeviceArray(n, np.uint8), ecc.DeviceArray(1, np.int32)
    gpu.kmeans_f32_engine(dev(ecc, f), n, d_c, ecc.kmeans_cfg(k=16, max_iters=3, tol=-1.0), engine, d_lab, d_it)
    gpu.sync()
    assert d_it.numpy()[0] == o_it
    assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32))
    assert (d_lab.numpy() == o_lab).all()


# ------------------------------------------------------------------------------ multi-GPU building blocks
def test_split_kmeans_equals_fused(ecc, orc, gpu):
    """accumulate -> (all-reduce) -> update, with two 'shards' summed on one device, equals the
    fused single-device loop bit for bit (integer partial sums)."""
    xy, rep_xy, u = _reps(ecc, orc, n=300_000, seed=13)
    nw = len(u)
    half = nw // 2
    k, iters = 16, 7
    c0 = _init_centroids(k, 9)
    o_c, o_lab, _ = orc.kmeans_run_xy16(np.concatenate([rep_xy[w * 8192: w * 8192 + u[w]] for w in range(nw)]), c0, iters)
    d_rep, d_u = dev(ecc, rep_xy), dev(ecc, u)
    d_c = dev(ecc, c0)
    acc = ecc.DeviceArray.zeros(3 * k, np.uint64)
    st = ecc.DeviceArray.zeros(2, np.int32)
    L = ecc.lib
    for _ in range(iters):
        # shard A = windows [0, half), shard B = windows [half, nw): same accumulator == all-reduce SUM
        ecc.check(L.ecc_kmeans_accumulate_xy16(gpu.ctx, d_rep.ptr, half, 8192, d_u.ptr, d_c.ptr, k, 50.0, acc.ptr, st.ptr, gpu.stream))
        ecc.check(L.ecc_kmeans_accumulate_xy16(gpu.ctx, d_rep.ptr + half * 8192 * 4, nw - half, 8192, d_u.ptr + half * 4,
                                               d_c.ptr, k, 50.0, acc.ptr, st.ptr, gpu.stream))
        ecc.check(L.ecc_kmeans_update(gpu.ctx, acc.ptr, d_c.ptr, k, -1.0, st.ptr, gpu.stream))
    lab = ecc.DeviceArray(nw * 8192, np.uint8)
    ecc.check(L.ecc_kmeans_labels_xy16(gpu.ctx, d_rep.ptr, nw, 8192, d_u.ptr, d_c.ptr, k, 50.0, lab.ptr, gpu.stream))
    gpu.sync()
    assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32))
    g = lab.numpy()
    assert (np.concatenate([g[w * 8192: w * 8192 + u[w]] for w in range(nw)]) == o_lab).all()
    assert st.numpy()[1] == iters


def test_sae_handoff_equals_single_stream(ecc, orc, gpu):
    """Shard the stream in 3 time windows: local SAEs -> max over lower shards -> detection per
    shard == detection over the whole stream."""
    W, H = W_SMALL, H_SMALL
    n = 16384 * 9
    xy, t, _ = ecc.gen_events(n, seed=17)
    o_flags, o_sae = orc.fast_detect(xy, t, W, H)
    shards = [(0, 16384 * 3), (16384 * 3, 16384 * 6), (16384 * 6, n)]
    imgs = ecc.DeviceArray.zeros(len(shards) * W * H, np.int64)
    for i, (lo, hi) in enumerate(shards):
        d_xy, d_t = dev(ecc, xy[lo:hi]), dev(ecc, t[lo:hi])  # keep alive until the launch completes
        ecc.check(ecc.lib.ecc_sae_scatter(gpu.ctx, d_xy.ptr, d_t.ptr, hi - lo, W, H,
                                          imgs.ptr + i * W * H * 8, gpu.stream))
        gpu.sync()
    flags = []
    for i, (lo, hi) in enumerate(shards):
        base = ecc.DeviceArray(W * H, np.int64)
        ecc.check(ecc.lib.ecc_sae_max_combine(gpu.ctx, imgs.ptr, i, W * H, base.ptr, gpu.stream))
        f, _ = _fast_gpu(ecc, gpu, xy[lo:hi], t[lo:hi], W, H, first_detect=1 if i == 0 else 0, sae0=base.numpy())
        flags.append(f)
    assert (np.concatenate(flags) == o_flags).all()


# ------------------------------------------------------------------------------ DBSCAN extraction (§8f rank 3)
def _dbscan_gpu(ecc, gpu, xy, n_segs, stride, counts, eps, min_pts, min_size, max_size, fused=False):
    d_xy = dev(ecc, xy)
    d_u = None if counts is None else dev(ecc, counts)
    n = n_segs * stride
    if fused:  # ecc_dbscan_grid: no neighbour lists
        d_lab = ecc.DeviceArray(n, np.int32)
        d_nc = ecc.DeviceArray(n_segs, np.int32)
        dup_cap = 1 << 20
        d_dups = ecc.DeviceArray(2 * dup_cap, np.int64)
        d_nd = ecc.DeviceArray(1, np.int64)
        gpu.dbscan_grid(d_xy, n_segs, stride, d_u, eps, min_pts, min_size, max_size, d_lab, d_nc, d_dups,
                        dup_cap, d_nd)
        return _dbscan_collect(ecc, gpu, n_segs, stride, counts, d_lab, d_nc, d_dups, d_nd)
    d_cnt = ecc.DeviceArray(n, np.int32)
    gpu.eps_counts(d_xy, n_segs, stride, d_u, eps, 1, d_cnt, None)
    d_off = ecc.DeviceArray(n + 1, np.int64)
    gpu.sync()
    cnt = d_cnt.numpy()
    valid = np.zeros(n, bool)
    for s in range(n_segs):
        valid[s * stride: s * stride + (stride if counts is None else counts[s])] = True
    cap = int(cnt[valid].sum()) + 16
    d_nbr = ecc.DeviceArray(cap, np.int32)
    gpu.eps_lists(d_xy, n_segs, stride, d_u, eps, d_cnt, d_off, d_nbr, cap)
    total = C.c_int64(0)
    ecc.check(ecc.lib.ecc_eps_total(gpu.ctx, d_off.ptr, n, C.byref(total), gpu.stream))
    assert total.value <= cap
    d_lab = ecc.DeviceArray(n, np.int32)
    d_nc = ecc.DeviceArray(n_segs, np.int32)
    dup_cap = 1 << 20
    d_dups = ecc.DeviceArray(2 * dup_cap, np.int64)
    d_nd = ecc.DeviceArray(1, np.int64)
    gpu.dbscan_extract(n_segs, stride, d_u, d_off, d_nbr, min_pts, min_size, max_size, d_lab, d_nc, d_dups,
                       dup_cap, d_nd)
    return _dbscan_collect(ecc, gpu, n_segs, stride, counts, d_lab, d_nc, d_dups, d_nd)


def _dbscan_collect(ecc, gpu, n_segs, stride, counts, d_lab, d_nc, d_dups, d_nd):
    st = gpu.dbscan_status()
    assert st == 0, gpu.last_error()
    lab, nc, nd = d_lab.numpy(), d_nc.numpy(), int(d_nd.numpy()[0])
    dups = d_dups.numpy()[:2 * nd].reshape(-1, 2)
    out = []
    for s in range(n_segs):
        m = stride if counts is None else counts[s]
        members = [[] for _ in range(nc[s])]
        for j in range(m):
            if lab[s * stride + j] >= 0:
                members[lab[s * stride + j]].append(j)
        for p, c in dups[(dups[:, 0] >= s * stride) & (dups[:, 0] < s * stride + m)]:
            members[c].append(int(p - s * stride))
        out.append([np.array(sorted(c), np.int32) for c in members])
    return out


@pytest.mark.parametrize("fused", [False, True], ids=["lists", "grid"])
@pytest.mark.parametrize("eps,min_pts,min_size,max_size", [
    (20.0, 20, 100, 25000),   # pcl_cluster.cpp:113-120 driver parameters
    (3.0, 4, 1, 1 << 30),
    (1.5, 3, 2, 50),
])
def test_dbscan_extract_matches_reference_semantics(ecc, orc, gpu, eps, min_pts, min_size, max_size, fused):
    xy, _, _ = ecc.gen_events(40_000, seed=61)
    rep_xy, _, u, _ = orc.downsample_hash(xy)
    nw = min(len(u), 4)
    got = _dbscan_gpu(ecc, gpu, rep_xy[:nw * 8192], nw, 8192, u[:nw], eps, min_pts, min_size, max_size, fused)
    for w in range(nw):
        pts = rep_xy[w * 8192: w * 8192 + u[w]]
        ref = orc.dbscan_lists(np.stack([pts & 0xFFFF, pts >> 16], 1), eps, min_pts, min_size, max_size)
        assert len(got[w]) == len(ref)
        for a, b in zip(got[w], ref):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("fused", [False, True], ids=["lists", "grid"])
def test_dbscan_extract_border_duplicates(ecc, orc, gpu, fused):
    """Many tiny random segments (dense in seeds, borders and duplicate memberships)."""
    rng = np.random.default_rng(7)
    n_segs, stride = 300, 64
    counts = rng.integers(1, stride + 1, n_segs).astype(np.int32)
    xy = ecc.pack_xy(rng.integers(0, 14, n_segs * stride), rng.integers(0, 14, n_segs * stride))
    got = _dbscan_gpu(ecc, gpu, xy, n_segs, stride, counts, 2.0, 4, 1, 1 << 30, fused)
    n_dup = 0
    for s in range(n_segs):
        pts = xy[s * stride: s * stride + counts[s]]
        ref = orc.dbscan_lists(np.stack([pts & 0xFFFF, pts >> 16], 1), 2.0, 4)
        assert len(got[s]) == len(ref), s
        for a, b in zip(got[s], ref):
            assert np.array_equal(a, b), s
        n_dup += sum(len(c) for c in ref) - len(set(np.concatenate(ref).tolist())) if ref else 0
    assert n_dup > 0  # the case really exercises duplicate memberships


@pytest.mark.parametrize("eps,min_pts", [(1.0, 2), (1.5, 3), (2.0, 4), (3.7, 6), (6.0, 12), (12.5, 30), (40.0, 50)])
@pytest.mark.parametrize("path", ["run", "grid_only"])
def test_dbscan_grid_distinct_pixel_segments(ecc, orc, gpu, monkeypatch, eps, min_pts, path):
    """Segments of DISTINCT pixels (the downsample windows' case: ecc_dbscan_grid's row-run kernel)
    mixed with segments that repeat a pixel (left to the cell-grid kernel) in one call: dense
    random patches with holes (chains broken inside chords, border points reached by several
    seeds), sparse scatter, a full square, a single row and column, one and zero points — against
    the oracle's literal seed queue.  `grid_only` forces the cell-grid kernel for every segment."""
    if path == "grid_only":
        monkeypatch.setenv("ECC_DBSCAN_GRID_ONLY", "1")
    rng = np.random.default_rng(int(eps * 10) + min_pts)
    stride = 2048
    segs = []
    for k in range(40):
        kind = k % 8
        if kind == 0:    # dense patch with holes
            side = int(rng.integers(20, 60))
            cells = rng.choice(side * side, int(side * side * rng.uniform(0.2, 0.7)), replace=False)
            pts = np.stack([cells % side, cells // side], 1) + rng.integers(0, 200, 2)
        elif kind == 1:  # sparse scatter over a large box
            cells = rng.choice(300 * 250, int(rng.integers(50, 2000)), replace=False)
            pts = np.stack([cells % 300, cells // 300], 1)
        elif kind == 2:  # a full square
            side = int(rng.integers(3, 40))
            g = np.arange(side * side)
            pts = np.stack([g % side, g // side], 1) + 5
        elif kind == 3:  # one row and one column with gaps
            xs = np.unique(rng.integers(0, 340, 300))
            pts = np.concatenate([np.stack([xs, np.full_like(xs, 7)], 1), np.stack([np.full_like(xs[:200], 11), xs[:200] % 250], 1)])
            pts = np.unique(pts, axis=0)
        elif kind == 4:  # repeats a pixel: the cell-grid kernel's segment
            pts = rng.integers(0, 30, (int(rng.integers(10, 800)), 2))
        elif kind == 5:
            pts = rng.integers(0, 346, (1, 2))
        elif kind == 6:
            pts = np.zeros((0, 2), np.int64)
        else:            # clustered blobs of distinct pixels
            c = rng.integers(20, 300, (6, 2))
            raw = (c[rng.integers(0, 6, 3000)] + rng.normal(0, eps * 1.5, (3000, 2))).round().astype(np.int64)
            raw = np.clip(raw, 0, 345)
            pts = np.unique(raw, axis=0)
            pts = pts[rng.permutation(len(pts))]
        pts = pts[:stride]
        if kind not in (4,):
            pts = pts[rng.permutation(len(pts))]
        segs.append(pts.astype(np.int64))
    counts = np.array([len(p) for p in segs], np.int32)
    xy = np.zeros(len(segs) * stride, np.uint32)
    for s, p in enumerate(segs):
        if len(p):
            xy[s * stride: s * stride + len(p)] = ecc.pack_xy(p[:, 0], p[:, 1])
    got = _dbscan_gpu(ecc, gpu, xy, len(segs), stride, counts, eps, min_pts, 1, 1 << 30, True)
    for s, p in enumerate(segs):
        ref = orc.dbscan_lists(p.reshape(-1, 2), eps, min_pts) if len(p) else []
        assert len(got[s]) == len(ref), (s, len(got[s]), len(ref))
        for a, b in zip(got[s], ref):
            assert np.array_equal(a, b), s


@pytest.mark.parametrize("n_comp", [1023, 1024, 1025, 2000])
def test_dbscan_grid_many_components(ecc, orc, gpu, n_comp):
    """Distinct-pixel segments with about kDrComp (1 024) components: isolated lattice points at
    min_pts 1 (every point a core point and its own cluster) plus a few two-point clusters.  Up to
    1 024 the row-run kernel keeps the segment; above, it leaves it to the cell-grid kernel, whose
    tables hold 4 096 — the output must be the oracle's either way."""
    rng = np.random.default_rng(n_comp)
    stride = 4096
    segs = []
    for k in range(3):
        g = rng.permutation(170 * 130)[:n_comp]
        pts = np.stack([(g % 170) * 2, (g // 170) * 2], 1)  # spacing 2 > eps: isolated
        if k == 1:  # some pairs: a neighbour at distance 1 joins a lattice point's cluster
            pts = np.concatenate([pts, pts[:50] + [1, 0]])
        segs.append(pts[rng.permutation(len(pts))].astype(np.int64))
    counts = np.array([len(p) for p in segs], np.int32)
    xy = np.zeros(len(segs) * stride, np.uint32)
    for s, p in enumerate(segs):
        xy[s * stride: s * stride + len(p)] = ecc.pack_xy(p[:, 0], p[:, 1])
    got = _dbscan_gpu(ecc, gpu, xy, len(segs), stride, counts, 1.0, 1, 1, 1 << 30, True)
    for s, p in enumerate(segs):
        ref = orc.dbscan_lists(p.reshape(-1, 2), 1.0, 1)
        assert len(got[s]) == len(ref), (s, len(got[s]), len(ref))
        for a, b in zip(got[s], ref):
            assert np.array_equal(a, b), s


def test_dbscan_extract_rejects_short_lists(ecc, gpu):
    """offsets that run past nbr_len: the segment is rejected (status CAPACITY), never read."""
    n = 64
    d_off = dev(ecc, np.arange(n + 1, dtype=np.int64) * 10)    # claims 640 entries
    d_nbr = dev(ecc, np.zeros(100, np.int32))                  # holds 100
    d_lab = ecc.DeviceArray(n, np.int32)
    d_nc = ecc.DeviceArray(1, np.int32)
    d_nd = ecc.DeviceArray(1, np.int64)
    gpu.dbscan_extract(1, n, None, d_off, d_nbr, 3, 1, 1 << 30, d_lab, d_nc, None, 0, d_nd)
    assert gpu.dbscan_status() == ecc.ERR_CAPACITY
    assert (d_lab.numpy() == -1).all() and int(d_nc.numpy()[0]) == 0


def test_dbscan_extract_rejects_out_of_segment_neighbours(ecc, gpu):
    """A list entry outside [0, m) is never used as an LDS index: status INVALID; a good call
    afterwards is OK again."""
    m, stride = 40, 64
    lists = [[j, (j + 1) % m] for j in range(m)]
    lists[7].append(m + 3)       # past the segment's points, inside the stride
    lists[9].append(100000)      # far outside
    lists[11].append(-5)
    off = np.zeros(stride + 1, np.int64)
    off[1:m + 1] = np.cumsum([len(l) for l in lists])
    off[m + 1:] = off[m]
    nbr = np.concatenate([np.array(l, np.int32) for l in lists])
    d_off, d_nbr = dev(ecc, off), dev(ecc, nbr)
    d_cnt = dev(ecc, np.array([m], np.int32))
    d_lab, d_nc, d_nd = ecc.DeviceArray(stride, np.int32), ecc.DeviceArray(1, np.int32), ecc.DeviceArray(1, np.int64)
    gpu.dbscan_extract(1, stride, d_cnt, d_off, d_nbr, 2, 1, 1 << 30, d_lab, d_nc, None, 0, d_nd)
    assert gpu.dbscan_status() == ecc.ERR_INVALID
    good = np.concatenate([np.array(l[:2], np.int32) for l in lists])
    off[1:m + 1] = np.arange(1, m + 1) * 2
    off[m + 1:] = off[m]
    d_off, d_nbr = dev(ecc, off), dev(ecc, good)
    gpu.dbscan_extract(1, stride, d_cnt, d_off, d_nbr, 2, 1, 1 << 30, d_lab, d_nc, None, 0, d_nd)
    assert gpu.dbscan_status() == 0
    assert int(d_nc.numpy()[0]) == 1 and (d_lab.numpy()[:m] == 0).all()  # one ring of 40 core points


# ------------------------------------------------------------------------------ HIP graph replay
def test_graph_replay_matches_eager(ecc, orc, gpu):
    """ecc_graph_begin/end/launch: a captured downsample -> k-means -> corners -> NMS step replays
    to the same outputs as the eager calls (and as the oracle's corner flags)."""
    W, H = 346, 260
    n = 16384 * 40
    xy, t, _ = ecc.gen_events(n, seed=77, width=W, height=H)
    d_xy, d_t = dev(ecc, xy), dev(ecc, t)
    n_win = (n + 8191) // 8192
    hcfg = ecc.hash_cfg(window=8192)
    rep_xy, uniq, rep = ecc.DeviceArray(n_win * 8192, np.uint32), ecc.DeviceArray(n_win, np.int32), ecc.DeviceArray(n_win, np.int32)
    K = 16
    c0 = np.stack([np.linspace(20, W - 20, K), np.linspace(20, H - 20, K)[::-1]], 1).astype(np.float32).ravel()
    d_c0, d_c = dev(ecc, c0), ecc.DeviceArray(2 * K, np.float32)
    labels = ecc.DeviceArray(n_win * 8192, np.uint8)
    kcfg = ecc.kmeans_cfg(k=K, max_iters=5, tol=-1.0)
    ccfg = ecc.corner_cfg(width=W, height=H)
    sae, flags = ecc.DeviceArray(W * H, np.int64), ecc.DeviceArray(n, np.uint8)
    ns, cap = n // 16384, 4096
    nms_out, nms_cnt = ecc.DeviceArray(ns * cap, ecc.CORNER_DTYPE), ecc.DeviceArray(ns, np.int32)
    lib = ecc.lib

    def step():
        ecc.check(lib.ecc_downsample_hash(gpu.ctx, d_xy.ptr, n, ecc.C.byref(hcfg), rep_xy.ptr, None, uniq.ptr,
                                          rep.ptr, gpu.stream))
        ecc.check(lib.ecc_memcpy_d2d(d_c.ptr, d_c0.ptr, 8 * K, gpu.stream))
        gpu.kmeans_xy16(rep_xy, n_win, 8192, uniq, d_c, kcfg, labels)
        ecc.check(lib.ecc_memset_async(sae.ptr, 0, sae.nbytes, gpu.stream))
        gpu.fast_detect(d_xy, d_t, n, ccfg, sae, flags)
        gpu.corner_nms(d_xy, flags, n, 16384, W, H, 15, cap, nms_out, nms_cnt)

    step()
    gpu.sync()
    eager = [a.numpy().copy() for a in (rep_xy, d_c, labels, sae, flags, nms_cnt)]
    o_flags, _ = orc.fast_detect(xy, t, W, H)
    assert (eager[4] == o_flags).all()
    gp = ecc.P()
    ecc.check(lib.ecc_graph_begin(gpu.stream))
    step()
    ecc.check(lib.ecc_graph_end(gpu.stream, ecc.C.byref(gp)))
    for a in (rep_xy, d_c, labels, sae, flags, nms_cnt):  # poison the outputs, then replay twice
        ecc.check(lib.ecc_memset_async(a.ptr, 0xA5, a.nbytes, gpu.stream))
    for _ in range(2):
        ecc.check(lib.ecc_graph_launch(gp.value, gpu.stream))
    gpu.sync()
    ecc.check(lib.ecc_graph_destroy(gp.value))
    u = uniq.numpy()
    valid = (np.arange(8192)[None, :] < u[:, None]).ravel()  # written slots of the windowed outputs
    for e, a, windowed in zip(eager, (rep_xy, d_c, labels, sae, flags, nms_cnt), (1, 0, 1, 0, 0, 0)):
        got = a.numpy()
        assert (got[valid] == e[valid]).all() if windowed else (got == e).all()


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [2, 3, 5])
def test_corner_shards_in_one_device_equal_one_call(ecc, orc, gpu, parts):
    """Time-window shards on separate contexts and streams of ONE device (bench.py
    --corner-shards): prepare each shard, start shard p from ecc_sae_max_combine of the lower
    shards' own last images, ecc_fast_detect_finish_nms — flags, final SAE and NMS lists equal the
    one-call ecc_fast_detect_nms and the oracle (Q15 only on the first shard)."""
    W, H = 346, 260
    ns = 67  # slices; uneven cuts, shards of different group alignment
    n = ns * 16384
    xy, t, _ = ecc.gen_events(n, seed=17, width=W, height=H)
    d_xy, d_t = dev(ecc, xy), dev(ecc, t)
    cap, HW = 2048, W * H
    flags, sae = ecc.DeviceArray(n, np.uint8), ecc.DeviceArray(HW, np.int64)
    out, cnt = ecc.DeviceArray(ns * cap, ecc.CORNER_DTYPE), ecc.DeviceArray(ns, np.int32)
    sae.fill_bytes(0, gpu.stream)
    gpu.fast_detect_nms(d_xy, d_t, n, ecc.corner_cfg(width=W, height=H), sae, flags, 15, cap, out, cnt)
    gpu.sync()
    ref = [a.numpy() for a in (flags, sae, out, cnt)]
    o_flags, o_sae = orc.fast_detect(xy, t, W, H)
    assert (ref[0] == o_flags).all() and (ref[1] == o_sae).all()
    lib = ecc.lib
    cuts = [round(p * ns / parts) * 16384 for p in range(parts + 1)]
    ctxs = [gpu] + [ecc.Context(0) for _ in range(parts - 1)]
    last = ecc.DeviceArray(parts * HW, np.int64)
    saes = [ecc.DeviceArray(HW, np.int64) for _ in range(parts)]
    f2, o2, c2 = ecc.DeviceArray(n, np.uint8), ecc.DeviceArray(ns * cap, ecc.CORNER_DTYPE), ecc.DeviceArray(ns, np.int32)
    f2.fill_bytes(0xA5, gpu.stream)
    cfgs = [ecc.corner_cfg(width=W, height=H, first_detect_slice=1 if p == 0 else 0) for p in range(parts)]
    evs = []
    for p in range(parts):
        e = ecc.P()
        ecc.check(lib.ecc_event_create(ecc.C.byref(e)))
        evs.append(e)
    gpu.sync()
    for p, cx in enumerate(ctxs):
        lo, m = cuts[p], cuts[p + 1] - cuts[p]
        ecc.check(lib.ecc_fast_detect_prepare(cx.ctx, d_xy.ptr + 4 * lo, d_t.ptr + 8 * lo, m, ecc.C.byref(cfgs[p]),
                                              last.ptr + 8 * p * HW, cx.stream))
        ecc.check(lib.ecc_event_record(evs[p], cx.stream))
    for p, cx in enumerate(ctxs):
        lo, m = cuts[p], cuts[p + 1] - cuts[p]
        for q in range(p):
            ecc.check(lib.ecc_stream_wait_event(cx.stream, evs[q]))
        ecc.check(lib.ecc_sae_max_combine(cx.ctx, last.ptr, p, HW, saes[p].ptr, cx.stream))
        s0 = lo // 16384
        ecc.check(lib.ecc_fast_detect_finish_nms(cx.ctx, d_xy.ptr + 4 * lo, d_t.ptr + 8 * lo, m, ecc.C.byref(cfgs[p]),
                                                 saes[p].ptr, f2.ptr + lo, 15, cap,
                                                 o2.ptr + s0 * cap * ecc.CORNER_DTYPE.itemsize, c2.ptr + 4 * s0,
                                                 cx.stream))
    for cx in ctxs:
        cx.sync()
        assert cx.fast_detect_status() == 0 and cx.corner_nms_status() == 0
    assert (f2.numpy() == ref[0]).all()
    assert (saes[-1].numpy() == ref[1]).all()
    c = c2.numpy()
    assert (c == ref[3]).all()
    got, want = o2.numpy(), ref[2]
    for s in range(ns):
        assert (got[s * cap: s * cap + c[s]] == want[s * cap: s * cap + c[s]]).all(), s
    for cx in ctxs[1:]:
        cx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("with_nms", [False, True])
def test_graph_replay_reports_unsorted_time_per_replay(ecc, gpu, with_nms):
    """The unsorted-time verdict is produced inside the captured work: a replay over unsorted
    timestamps reports ECC_ERR_UNSORTED_TIME, the next replay over sorted ones reports OK, and an
    eager call between replays does not leak its verdict into them."""
    W, H = 346, 260
    n = 16384 * 6
    xy, t, _ = ecc.gen_events(n, seed=5, width=W, height=H)
    bad_t = t.copy()
    bad_t[n // 2], bad_t[n // 2 + 1] = t[n // 2 + 1] + 5, t[n // 2]
    d_xy, d_t = dev(ecc, xy), dev(ecc, t)
    d_tbad, d_tok = dev(ecc, bad_t), dev(ecc, t)
    ccfg = ecc.corner_cfg(width=W, height=H)
    sae, flags = ecc.DeviceArray(W * H, np.int64), ecc.DeviceArray(n, np.uint8)
    ns, cap = n // 16384, 1024
    out, cnt = ecc.DeviceArray(ns * cap, ecc.CORNER_DTYPE), ecc.DeviceArray(ns, np.int32)
    lib = ecc.lib

    def detect(tt):
        if with_nms:
            gpu.fast_detect_nms(d_xy, tt, n, ccfg, sae, flags, 15, cap, out, cnt)
        else:
            gpu.fast_detect(d_xy, tt, n, ccfg, sae, flags)

    detect(d_t)
    gpu.sync()
    assert gpu.fast_detect_status() == 0
    gp = ecc.P()
    ecc.check(lib.ecc_graph_begin(gpu.stream))
    detect(d_t)
    ecc.check(lib.ecc_graph_end(gpu.stream, ecc.C.byref(gp)))
    unsorted = ecc.ERR_UNSORTED_TIME
    try:
        for t_src, want in ((bad_t, unsorted), (t, 0), (bad_t, unsorted), (bad_t, unsorted), (t, 0)):
            ecc.check(lib.ecc_memcpy_h2d(d_t.ptr, t_src.ctypes.data, t_src.nbytes, gpu.stream))
            ecc.check(lib.ecc_graph_launch(gp.value, gpu.stream))
            gpu.sync()
            assert gpu.fast_detect_status() == want, (want, t_src is bad_t)
        # an eager unsorted call, then a sorted replay: OK; an eager sorted call, then an
        # unsorted replay: the error
        detect(d_tbad)
        gpu.sync()
        assert gpu.fast_detect_status() == unsorted
        ecc.check(lib.ecc_graph_launch(gp.value, gpu.stream))  # d_t holds the sorted t
        gpu.sync()
        assert gpu.fast_detect_status() == 0
        ecc.check(lib.ecc_memcpy_h2d(d_t.ptr, bad_t.ctypes.data, bad_t.nbytes, gpu.stream))
        detect(d_tok)
        gpu.sync()
        assert gpu.fast_detect_status() == 0
        ecc.check(lib.ecc_graph_launch(gp.value, gpu.stream))
        gpu.sync()
        assert gpu.fast_detect_status() == unsorted
    finally:
        ecc.check(lib.ecc_graph_destroy(gp.value))


# ------------------------------------------------------------------------------ multi-GPU forms
def test_fast_detect_prepare_finish_matches_one_call(ecc, orc, gpu):
    """prepare (sort + pair entries + the batch's own last-t image) then finish (from a given
    initial SAE) == ecc_fast_detect; the last-t image == per-pixel max t of the batch."""
    W, H = 346, 260
    n = 16384 * 45 + 1234
    xy, t, _ = ecc.gen_events(n, seed=91, width=W, height=H)
    sae0 = np.zeros(W * H, np.int64)
    sae0[::7] = 5  # a non-trivial initial surface
    o_flags, o_sae = orc.fast_detect(xy, t, W, H, first_detect=0, sae=sae0.copy())
    cfg = ecc.corner_cfg(width=W, height=H, first_detect_slice=0)
    d_xy, d_t = dev(ecc, xy), dev(ecc, t)
    local = ecc.DeviceArray(W * H, np.int64)
    sae, flags = dev(ecc, sae0), ecc.DeviceArray(n, np.uint8)
    lib = ecc.lib
    ecc.check(lib.ecc_fast_detect_prepare(gpu.ctx, d_xy.ptr, d_t.ptr, n, ecc.C.byref(cfg), local.ptr, gpu.stream))
    ecc.check(lib.ecc_fast_detect_finish(gpu.ctx, d_xy.ptr, d_t.ptr, n, ecc.C.byref(cfg), sae.ptr, flags.ptr,
                                         gpu.stream))
    assert gpu.fast_detect_status() == 0
    assert (flags.numpy() == o_flags).all()
    assert (sae.numpy() == o_sae).all()
    x, y = ecc.unpack_xy(xy)
    ref = np.zeros(W * H, np.int64)
    np.maximum.at(ref, y.astype(np.int64) * W + x, t)
    assert (local.numpy() == ref).all()


def test_kmeans_count_images_sum_over_shards(ecc, orc, gpu):
    """Two shards' per-pixel count images, summed, then ecc_kmeans_run_counts == the oracle's
    k-means over the union of the shards' points (bit-identical centroids)."""
    W, H, K = 346, 260, 16
    xy, _, _ = ecc.gen_events(16384 * 30, seed=33, width=W, height=H)
    rx, _, u, _ = orc.downsample_hash(xy)
    pts = np.concatenate([rx[w * 8192: w * 8192 + u[w]] for w in range(len(u))])
    half = len(pts) // 2
    c0 = np.stack([np.linspace(20, W - 20, K), np.linspace(20, H - 20, K)[::-1]], 1).astype(np.float32).ravel()
    lib = ecc.lib
    total = np.zeros(W * H, np.uint32)
    for part in (pts[:half], pts[half:]):
        cnt = ecc.DeviceArray(W * H, np.uint32)
        ecc.check(lib.ecc_kmeans_counts_xy16(gpu.ctx, dev(ecc, part).ptr, 1, len(part), None, W, H, cnt.ptr,
                                             gpu.stream))
        assert lib.ecc_kmeans_counts_status(gpu.ctx, gpu.stream) == 0
        total += cnt.numpy()
    xs, ys = ecc.unpack_xy(pts)
    assert (total == np.bincount(ys.astype(np.int64) * W + xs, minlength=W * H)).all()
    kcfg = ecc.kmeans_cfg(k=K, max_iters=10, tol=-1.0)
    d_c = dev(ecc, c0)
    ecc.check(lib.ecc_kmeans_run_counts(gpu.ctx, dev(ecc, total).ptr, W, H, ecc.C.byref(kcfg), d_c.ptr, None,
                                        gpu.stream))
    gpu.sync()
    o_c, _, _ = orc.kmeans_run_xy16(pts, c0, 10)
    assert np.array_equal(d_c.numpy().view(np.uint32), o_c.view(np.uint32))
    # a point outside the frame is reported
    bad = np.array([ecc.pack_xy(W, 3)], np.uint32)
    cnt = ecc.DeviceArray(W * H, np.uint32)
    ecc.check(lib.ecc_kmeans_counts_xy16(gpu.ctx, dev(ecc, bad).ptr, 1, 1, None, W, H, cnt.ptr, gpu.stream))
    assert lib.ecc_kmeans_counts_status(gpu.ctx, gpu.stream) == ecc.ERR_INVALID


@pytest.mark.parametrize("case", ["hot", "chunks", "segments"])
def test_kmeans_count_images_exact(ecc, gpu, case):
    """Per-pixel count images against np.bincount where the chunked LDS counts are hardest: one
    pixel holding more than 2^16 points of one part, frames of many 32 K-pixel chunks with points
    at the chunk edges and the frame's corners, and ragged segments (each call made twice: no
    state leaks between calls)."""
    rng = np.random.default_rng(7)
    if case == "hot":
        W, H = 346, 260
        n = 300_000
        x = np.where(rng.random(n) < 0.8, 5, rng.integers(0, W, n))
        y = np.where(x == 5, 7, rng.integers(0, H, n))
        segs, stride, counts = 1, n, None
    elif case == "chunks":
        W, H = 1280, 720  # 14 chunks of 65536 pixels
        n = 200_000
        idx = np.concatenate([rng.integers(0, W * H, n - 8), [0, W * H - 1, 65535, 65536, 131071, 131072, W - 1,
                                                               (H - 1) * W]])
        x, y = idx % W, idx // W
        segs, stride, counts = 1, n, None
    else:
        W, H = 346, 260
        segs, stride = 97, 4096
        counts = rng.integers(0, stride + 1, segs).astype(np.int32)
        n = segs * stride
        x, y = rng.integers(0, W, n), rng.integers(0, H, n)
    pts = ecc.pack_xy(x.astype(np.uint32), y.astype(np.uint32)).astype(np.uint32)
    if counts is None:
        ref = np.bincount(y.astype(np.int64) * W + x, minlength=W * H)
    else:
        valid = (np.arange(stride)[None, :] < counts[:, None]).ravel()
        ref = np.bincount((y.astype(np.int64) * W + x)[valid], minlength=W * H)
    d_pts = dev(ecc, pts)
    d_cnt = None if counts is None else dev(ecc, counts)
    lib = ecc.lib
    for _ in range(2):
        cnt = ecc.DeviceArray(W * H, np.uint32)
        ecc.check(lib.ecc_kmeans_counts_xy16(gpu.ctx, d_pts.ptr, segs, stride, None if d_cnt is None else d_cnt.ptr,
                                             W, H, cnt.ptr, gpu.stream))
        assert lib.ecc_kmeans_counts_status(gpu.ctx, gpu.stream) == 0
        assert (cnt.numpy() == ref).all(), np.nonzero(cnt.numpy() != ref)[0][:8]


# ------------------------------------------------------------------------------ fp64 radius / OPTICS
def _brute_ball(pts, i, eps2):
    """square_distance (kdTree.hpp:180-192) in the same operation order, vectorised."""
    s = np.zeros(len(pts))
    for d in range(pts.shape[1]):
        dd = pts[:, d] - pts[i, d]
        s = s + dd * dd
    return s <= eps2, s


@pytest.mark.parametrize("dim,n,eps,min_pts,kind", [
    (2, 3000, 0.02, 10, "uniform"), (3, 3000, 0.06, 10, "uniform"), (1, 2000, 0.001, 4, "uniform"),
    (2, 3000, 1.5, 20, "blobs"), (3, 2500, 2.0, 64, "blobs"), (2, 1500, 0.0, 1, "dups"),
])
def test_radius_f64_matches_brute_force(ecc, gpu, dim, n, eps, min_pts, kind):
    rng = np.random.default_rng(dim * 100 + n)
    if kind == "uniform":
        pts = rng.random((n, dim))
    elif kind == "blobs":
        pts = rng.normal(0, 3, (n, dim)) + rng.integers(0, 4, (n, 1)) * 25.0
    else:  # many exact duplicates (eps 0: the ball is the set of equal points)
        pts = rng.integers(0, 30, (n, dim)).astype(np.float64)
    d_pts = dev(ecc, pts)
    cnt = ecc.DeviceArray(n, np.int32)
    core = ecc.DeviceArray(n, np.float64)
    gpu.radius_counts_f64(d_pts, n, dim, eps, min_pts, cnt, core)
    off = ecc.DeviceArray(n + 1, np.int64)
    gpu.radius_lists_f64(d_pts, n, dim, eps, cnt, off, None, 0)
    gpu.sync()
    total = int(off.numpy()[n])
    nbr = ecc.DeviceArray(max(total, 1), np.int32)
    nd = ecc.DeviceArray(max(total, 1), np.float64)
    gpu.radius_lists_f64(d_pts, n, dim, eps, cnt, off, nbr, total, nd)
    gpu.sync()
    assert gpu.radius_status() == 0
    g_cnt, g_core, g_off, g_nbr, g_nd = cnt.numpy(), core.numpy(), off.numpy(), nbr.numpy(), nd.numpy()
    eps2 = eps * eps
    for i in range(n):
        ball, s = _brute_ball(pts, i, eps2)
        idx = np.nonzero(ball)[0]
        assert g_cnt[i] == len(idx), i
        lst = g_nbr[g_off[i]:g_off[i + 1]]
        assert sorted(lst.tolist()) == idx.tolist(), i
        assert np.array_equal(g_nd[g_off[i]:g_off[i + 1]], np.sqrt(s[lst])), i
        want = np.sqrt(np.sort(s[idx])[min_pts - 1]) if len(idx) >= min_pts else -1.0
        assert g_core[i] == want, (i, g_core[i], want)


def test_radius_f64_large_sampled(ecc, gpu):
    """500 000 uniform points (the published benchmark's size): counts of 2000 sampled points
    against brute force over all points; the list total equals the sum of the counts."""
    n, dim, eps = 500_000, 2, 0.0025
    rng = np.random.default_rng(5)
    pts = rng.random((n, dim))
    d_pts = dev(ecc, pts)
    cnt = ecc.DeviceArray(n, np.int32)
    gpu.radius_counts_f64(d_pts, n, dim, eps, 1, cnt, None)
    off = ecc.DeviceArray(n + 1, np.int64)
    gpu.radius_lists_f64(d_pts, n, dim, eps, cnt, off, None, 0)
    gpu.sync()
    g_cnt = cnt.numpy()
    assert int(off.numpy()[n]) == int(g_cnt.sum())
    for i in rng.choice(n, 2000, replace=False):
        ball, _ = _brute_ball(pts, i, eps * eps)
        assert g_cnt[i] == int(ball.sum()), i


@pytest.mark.parametrize("dim,n,min_pts,eps,kind", [
    (2, 2000, 10, -1.0, "uniform"), (3, 2000, 10, -1.0, "uniform"), (2, 1500, 5, 1.0, "blobs"),
    (1, 1000, 3, -1.0, "uniform"), (2, 1200, 2, 10.0, "pixels"),
])
def test_optics_f64_matches_oracle(ecc, orc, gpu, dim, n, min_pts, eps, kind):
    """The C ABI OPTICS (GPU eps-balls + host heap expansion) against the oracle's literal
    std::set expansion over brute-force balls: identical ordering and reachabilities."""
    rng = np.random.default_rng(n + dim)
    if kind == "uniform":
        pts = rng.random((n, dim))
    elif kind == "blobs":
        pts = rng.normal(0, 2, (n, dim)) + rng.integers(0, 5, (n, 1)) * 15.0
    else:  # integer pixels with duplicates (the event drivers' case, cluster_event_data.cpp)
        pts = rng.integers(0, 120, (n, dim)).astype(np.float64)
    g_order, g_reach = gpu.optics_f64(pts, min_pts, eps)
    o_order, o_reach = orc.optics(pts, min_pts, eps)
    assert np.array_equal(g_order, o_order)
    assert np.array_equal(g_reach.view(np.uint64), o_reach.view(np.uint64))
