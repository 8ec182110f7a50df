"""GPU parity of the any-size point-cloud paths (SURVEY.md §8a rows a9-a12 at the reference's own
input types), against the oracle's literal restatements:

* DBSCAN over float (x, y, z) clouds of any size — DBSCANSimpleCluster::extract with its
  brute-force radiusSearch (PCC/DBSCAN_simple.h:27-142, float per-axis differences widened to
  double) — on (x, y, t) event clouds above 25 000 points with the driver's eps 20 / minPts 20 /
  sizes 100..25000 (PCC/pcl_cluster.cpp:112-123), and DBSCANPrecompCluster (DBSCAN_precomp.h);
* eps-balls of fp32 clouds (counts, core distances, adjacency rows in ascending order);
* OPTICS core distances and orderings with min_pts above 64 (optics.hpp:286-299 has no cap).
"""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "event-camera-clustering-and-optical-flow-estimation_amd" / "bin"


def dev(ecc, a):
    return ecc.DeviceArray.from_numpy(np.ascontiguousarray(a))


def event_cloud(ecc, n, seed, t_scale, jitter=0.0):
    """(x, y, (t - t0) * t_scale) of a synthetic event stream as float32; `jitter` adds a fixed
    fractional offset pattern so that the coordinates are not integers."""
    xy, t, _ = ecc.gen_events(n, seed=seed)
    x, y = ecc.unpack_xy(xy)
    pts = np.stack([x, y, (t - t[0]) * t_scale], 1).astype(np.float64)
    if jitter:
        rng = np.random.default_rng(seed)
        pts += rng.uniform(-jitter, jitter, pts.shape)
    return pts.astype(np.float32)


def gpu_dbscan_cloud(ecc, gpu, pts, eps, min_pts, min_size, max_size, dup_cap=1 << 20):
    n, dim = pts.shape
    d_p = dev(ecc, pts.ravel())
    d_lab = ecc.DeviceArray(max(n, 1), np.int32)
    d_nc = ecc.DeviceArray(1, np.int32)
    d_dups = ecc.DeviceArray(2 * max(dup_cap, 1), np.int64)
    d_nd = ecc.DeviceArray(1, np.int64)
    gpu.dbscan_cloud(d_p, n, dim, eps, min_pts, min_size, max_size, d_lab, d_nc, d_dups, dup_cap, d_nd)
    st = gpu.dbscan_cloud_status()
    nd = int(d_nd.numpy()[0])
    if st == ecc.ERR_CAPACITY:
        return st, nd, None, None
    assert st == 0, gpu.last_error()
    lab, nc = d_lab.numpy()[:n], int(d_nc.numpy()[0])
    dups = d_dups.numpy()[:2 * nd].reshape(-1, 2)
    members = [[] for _ in range(nc)]
    for i in np.nonzero(lab >= 0)[0]:
        members[lab[i]].append(int(i))
    for p, c in dups:
        members[c].append(int(p))
    return st, nd, lab, [np.array(sorted(m), np.int32) for m in members]


def assert_same_clusters(got, ref):
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("t_scale,eps,min_pts,min_size,max_size,jitter", [
    (0.3, 20.0, 20, 100, 25000, 0.0),      # the driver's parameters on an (x, y, t) event cloud
    (0.3, 20.0, 20, 100, 25000, 0.45),     # non-integer float coordinates
    (0.01, 20.0, 20, 100, 25000, 0.0),     # one 29 998-point component: above max, filtered out
    (0.01, 20.0, 20, 100, 30000, 0.0),     # ... kept when max allows it (> 25 000 points)
    (1.0, 6.5, 5, 1, 1 << 30, 0.3),        # many small clusters, border duplicates
])
def test_dbscan_cloud_matches_reference_queue(ecc, orc, gpu, t_scale, eps, min_pts, min_size, max_size, jitter):
    pts = event_cloud(ecc, 30000, 11, t_scale, jitter)
    _, _, _, got = gpu_dbscan_cloud(ecc, gpu, pts, eps, min_pts, min_size, max_size)
    _, ref = orc.dbscan_cloud(pts, eps, min_pts, min_size, max_size)
    assert_same_clusters(got, ref)
    if max_size == 30000 and t_scale == 0.01:
        assert len(ref) == 1 and len(ref[0]) > 25000


def test_dbscan_cloud_float_difference_semantics(ecc, orc, gpu):
    """A pair whose float difference is within eps while the exact (double) one is not: the
    reference subtracts in float (DBSCAN_simple.h:132), so it is ONE cluster of two points."""
    rng = np.random.default_rng(5)
    eps = np.float64(20.0)
    found = None
    for _ in range(200000):
        a = np.float32(rng.uniform(-1, 1))
        b = np.float32(a - np.float32(20.0) - np.float32(rng.uniform(-4e-6, 4e-6)))
        fd = np.float64(np.float32(a - b))
        dd = np.float64(a) - np.float64(b)
        if fd * fd <= eps * eps < dd * dd:
            found = (a, b)
            break
    assert found is not None
    pts = np.array([[found[0], 0, 0], [found[1], 0, 0]], np.float32)
    _, ref = orc.dbscan_cloud(pts, float(eps), 2, 1, 10)
    assert len(ref) == 1 and len(ref[0]) == 2
    _, _, _, got = gpu_dbscan_cloud(ecc, gpu, pts, float(eps), 2, 1, 10)
    assert_same_clusters(got, ref)


def test_dbscan_cloud_f64_and_2d_agree_with_window_path(ecc, orc, gpu):
    """Integer 2-D points through the cloud path (fp64 and fp32, dims 2 and 3 with z = 0) equal
    the per-window extraction's reference lists."""
    xy, _, _ = ecc.gen_events(20000, seed=61)
    rep_xy, _, u, _ = orc.downsample_hash(xy)
    pts = rep_xy[:u[0]]
    p2 = np.stack([pts & 0xFFFF, pts >> 16], 1)
    ref = orc.dbscan_lists(p2, 3.0, 4)
    for cloud in (p2.astype(np.float64), p2.astype(np.float32),
                  np.concatenate([p2, np.zeros((len(p2), 1))], 1).astype(np.float32)):
        _, _, _, got = gpu_dbscan_cloud(ecc, gpu, cloud, 3.0, 4, 1, 1 << 30)
        assert_same_clusters(got, ref)


def test_dbscan_cloud_duplicate_capacity_and_edge_cases(ecc, orc, gpu):
    # 150 separate patches of 1..64 points on a 14x14 grid (eps 2, minPts 4): border points
    # reached by several seeds, i.e. duplicate memberships
    rng = np.random.default_rng(7)
    patches = []
    for k in range(150):
        m = int(rng.integers(1, 65))
        patches.append(rng.integers(0, 14, (m, 2)) + np.array([(k % 15) * 100, (k // 15) * 100]))
    pts = np.concatenate(patches).astype(np.float32)
    _, ref = orc.dbscan_cloud(pts, 2.0, 4)
    n_dup = sum(len(c) for c in ref) - len(set(np.concatenate(ref).tolist()))
    assert n_dup > 0
    st, nd, _, _ = gpu_dbscan_cloud(ecc, gpu, pts, 2.0, 4, 1, 1 << 30, dup_cap=0)
    assert st == ecc.ERR_CAPACITY and nd == n_dup
    _, _, _, got = gpu_dbscan_cloud(ecc, gpu, pts, 2.0, 4, 1, 1 << 30, dup_cap=nd)
    assert_same_clusters(got, ref)
    # a negative tolerance acts as |eps| (radius_square = radius * radius)
    _, _, _, got = gpu_dbscan_cloud(ecc, gpu, pts, -2.0, 4, 1, 1 << 30)
    assert_same_clusters(got, ref)
    # empty cloud, single point, all-identical points
    st, _, lab, got = gpu_dbscan_cloud(ecc, gpu, np.zeros((0, 3), np.float32), 1.0, 1, 1, 10)
    assert got == []
    _, _, lab, got = gpu_dbscan_cloud(ecc, gpu, np.ones((1, 3), np.float32), 1.0, 1, 1, 10)
    assert len(got) == 1 and list(got[0]) == [0]
    same = np.full((500, 3), 7.25, np.float32)
    _, _, _, got = gpu_dbscan_cloud(ecc, gpu, same, 0.0, 500, 1, 1 << 30)
    assert len(got) == 1 and len(got[0]) == 500


@pytest.mark.parametrize("min_pts", [1, 5])
def test_dbscan_cloud_non_finite_points_are_noise(ecc, orc, gpu, min_pts):
    """A point with a NaN or inf coordinate: `d2 <= r2` (DBSCAN_simple.h:132-136) is false for
    every pair with another point, but radiusSearch pushes the point itself unconditionally
    (:124-125), so it has one neighbour: noise for min_pts > 1, a singleton cluster for
    min_pts <= 1 (min size 1).  The rest is clustered as without it (a non-dense PCL cloud).
    Same here, with no error status, compared with the oracle's literal queue in every case — and
    a radius call in between does not change the status of the DBSCAN call before it."""
    pts = event_cloud(ecc, 8000, 31, 0.3, 0.45)
    rng = np.random.default_rng(3)
    bad = rng.choice(len(pts), 40, replace=False)
    vals = [np.nan, np.inf, -np.inf]
    for k, i in enumerate(bad):
        pts[i, k % 3] = vals[k % 3]
    pts[bad[0]] = np.nan  # all coordinates
    _, ref = orc.dbscan_cloud(pts, 6.0, min_pts, 1, 1 << 30)
    st, _, lab, got = gpu_dbscan_cloud(ecc, gpu, pts, 6.0, min_pts, 1, 1 << 30)
    assert st == 0
    assert_same_clusters(got, ref)
    assert len(got) > 5
    if min_pts > 1:
        assert (lab[bad] == -1).all()
    else:  # each non-finite point is a cluster of its own
        assert all(sum(1 for c in got if len(c) == 1 and c[0] == i) == 1 for i in bad)
    # an all-non-finite cloud: all noise, or all singletons at min_pts 1
    allbad = np.full((50, 3), np.nan, np.float32)
    allbad[::3, 1] = np.inf
    for mp, ms in ((1, 1), (5, 1), (1, 2)):
        _, ref = orc.dbscan_cloud(allbad, 1.0, mp, ms, 10)
        st, _, lab, got = gpu_dbscan_cloud(ecc, gpu, allbad, 1.0, mp, ms, 10)
        assert st == 0
        assert_same_clusters(got, ref)
        assert len(got) == (50 if (mp, ms) == (1, 1) else 0)
    # the radius path still reports non-finite input; DBSCAN's own status is its own word
    d_p = dev(ecc, pts.ravel())
    d_lab, d_nc, d_nd = ecc.DeviceArray(len(pts), np.int32), ecc.DeviceArray(1, np.int32), ecc.DeviceArray(1, np.int64)
    d_d = ecc.DeviceArray(2 << 20, np.int64)
    gpu.dbscan_cloud(d_p, len(pts), 3, 6.0, 5, 1, 1 << 30, d_lab, d_nc, d_d, 1 << 20, d_nd)
    cnt = ecc.DeviceArray(len(pts), np.int32)
    gpu.radius_counts_f32(d_p, len(pts), 3, 6.0, 0, cnt)
    assert gpu.radius_status() == ecc.ERR_INVALID
    assert gpu.dbscan_cloud_status() == 0


@pytest.mark.parametrize("min_pts", [1, 8, 64, 65, 100, 300])
def test_radius_f32_counts_core_lists_match_oracle(ecc, orc, gpu, min_pts):
    pts = event_cloud(ecc, 6000, 21, 0.05, 0.45)  # up to 218 neighbours: core points up to min_pts 100, none at 300
    n = len(pts)
    eps = 12.5
    o_cnt, o_core, o_off, o_nbr = orc.radius_f32(pts, eps, min_pts)
    d_p = dev(ecc, pts.ravel())
    d_cnt, d_core = ecc.DeviceArray(n, np.int32), ecc.DeviceArray(n, np.float64)
    gpu.radius_counts_f32(d_p, n, 3, eps, min_pts, d_cnt, d_core)
    assert np.array_equal(d_cnt.numpy(), o_cnt)
    assert np.array_equal(d_core.numpy().view(np.int64), o_core.view(np.int64))
    assert np.array_equal(o_core >= 0, o_cnt >= min_pts)
    if min_pts <= 100:  # the register network up to 64, the radix select above
        assert (o_core >= 0).any()
    if min_pts > 1:
        assert (o_core < 0).any()
    total = int(o_off[-1])
    d_off, d_nbr = ecc.DeviceArray(n + 1, np.int64), ecc.DeviceArray(total, np.int32)
    d_nd = ecc.DeviceArray(total, np.float64)
    gpu.radius_lists_f32(d_p, n, 3, eps, d_cnt, d_off, d_nbr, total, d_nd)
    gpu.lists_sort_ascending(n, d_off, total, d_nbr, d_nd)
    assert gpu.radius_status() == 0
    assert np.array_equal(d_off.numpy(), o_off)
    nbr, nd = d_nbr.numpy(), d_nd.numpy()
    assert np.array_equal(nbr, o_nbr[:total])
    # each distance travelled with its index: sqrt of the reference's d^2 for that pair
    i_of = np.repeat(np.arange(n), np.diff(o_off))
    diff = (pts[nbr] - pts[i_of]).astype(np.float64)  # float differences, widened
    d2 = diff[:, 0] * diff[:, 0] + diff[:, 1] * diff[:, 1] + diff[:, 2] * diff[:, 2]
    assert np.array_equal(nd, np.sqrt(d2))


@pytest.mark.parametrize("min_pts", [65, 100, 257])
def test_optics_min_pts_above_64_matches_oracle(ecc, orc, gpu, min_pts):
    rng = np.random.default_rng(min_pts)
    pts = np.concatenate([rng.normal(c, 1.0, (1500, 2)) for c in ([0, 0], [6, 2], [3, 9])])
    order, reach = gpu.optics_f64(pts, min_pts, 2.5)
    o_order, o_reach = orc.optics(pts, min_pts, 2.5)
    assert np.array_equal(order, o_order)
    assert np.array_equal(reach.view(np.int64), o_reach.view(np.int64))
    assert (reach > 0).sum() > 1000


def test_int_lists_beyond_16384_points_sorted_like_precomp(ecc, orc, gpu):
    """eps_neighbour_lists' path for more than 16384 points: the global grid (fp64, exact for
    int) + the segmented sort gives every row in ascending index order (DBSCAN_precomp.h)."""
    xy, _, _ = ecc.gen_events(60000, seed=3)
    rep_xy, _, u, _ = orc.downsample_hash(xy)
    pts = np.concatenate([rep_xy[w * 8192: w * 8192 + u[w]] for w in range(len(u))])[:20000]
    n = len(pts)
    assert n > 16384
    o_cnt, o_core, o_off, o_nbr = orc.eps_neighbours(pts, 1, n, None, 5.0, 90, want_lists=True)
    p2 = np.stack([pts & 0xFFFF, pts >> 16], 1).astype(np.float64)
    d_p = dev(ecc, p2.ravel())
    d_cnt, d_core = ecc.DeviceArray(n, np.int32), ecc.DeviceArray(n, np.float64)
    gpu.radius_counts_f64(d_p, n, 2, 5.0, 90, d_cnt, d_core)
    assert np.array_equal(d_cnt.numpy(), o_cnt)
    assert np.array_equal(d_core.numpy().view(np.int64), o_core.view(np.int64))
    total = int(o_off[-1])
    d_off, d_nbr = ecc.DeviceArray(n + 1, np.int64), ecc.DeviceArray(total, np.int32)
    gpu.radius_lists_f64(d_p, n, 2, 5.0, d_cnt, d_off, d_nbr, total)
    gpu.lists_sort_ascending(n, d_off, total, d_nbr)
    assert gpu.radius_status() == 0
    assert np.array_equal(d_off.numpy(), o_off)
    assert np.array_equal(d_nbr.numpy(), o_nbr[:total])


def _run(prog, *args):
    r = subprocess.run([str(BIN / prog)] + [str(a) for a in args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def _program_clusters(out):
    k = int(re.search(r"cluster size : (\d+)", out).group(1))
    rows = [l.split(",") for l in out.splitlines()[1:] if l.count(",") == 3]
    return k, rows


@pytest.mark.parametrize("variant", [[], ["--precomp"]])
def test_dbscan_program_event_cloud_xyt(ecc, orc, tmp_path, variant):
    """ecc_dbscan (the pcl_cluster.cpp driver) on an (x, y, t) event cloud of 30 000 events with
    its default eps 20 / minPts 20 / 100..25000: clusters and their member rows equal the oracle."""
    n, ts = 30000, 0.3
    xy, t, p = ecc.gen_events(n, seed=11)
    x, y = ecc.unpack_xy(xy)
    f = tmp_path / "e.csv"
    f.write_text("\n".join(f"{a},{b},{c},{d}" for a, b, c, d in zip(x, y, t - t[0], p)) + "\n")
    out = _run("ecc_dbscan", f, "--t-scale", ts, *variant)
    k, rows = _program_clusters(out)
    pts = np.stack([x, y, ((t - t[0]) * ts)], 1).astype(np.float32)
    _, ref = orc.dbscan_cloud(pts, 20.0, 20, 100, 25000)
    assert k == len(ref) and k > 3
    exp = [(float(pts[i, 0]), float(pts[i, 1]), float(pts[i, 2]), j % 8) for j, c in enumerate(ref) for i in c]
    got = [(float(a), float(b), float(c), int(d)) for a, b, c, d in rows]
    assert len(got) == len(exp)
    assert all(g[:2] == e[:2] and g[3] == e[3] and abs(g[2] - e[2]) <= 1e-4 * max(1.0, abs(e[2]))
               for g, e in zip(got, exp))


def test_dbscan_program_precomp_freezes_tolerance_at_input(ecc, orc, tmp_path):
    """DBSCANPrecompCluster::setInputCloud precomputes the adjacency with the tolerance set so far
    (DBSCAN_precomp.h:10-16, :28): input first, then eps 20 -> the eps-0 neighbourhoods."""
    xy, t, p = ecc.gen_events(4000, seed=12)
    x, y = ecc.unpack_xy(xy)
    f = tmp_path / "e.csv"
    f.write_text("\n".join(f"{a},{b},0,0" for a, b in zip(x, y)) + "\n")
    pts = np.stack([x, y, np.zeros_like(x)], 1).astype(np.float32)
    args = ["--min-pts", 2, "--min-size", 2, "--max-size", 100000]
    k_pre, rows_pre = _program_clusters(_run("ecc_dbscan", f, "--precomp", "--cloud-first", *args))
    _, ref0 = orc.dbscan_cloud(pts, 0.0, 2, 2, 100000)
    assert k_pre == len(ref0) and k_pre > 0
    k_simple, _ = _program_clusters(_run("ecc_dbscan", f, "--cloud-first", *args))
    _, ref20 = orc.dbscan_cloud(pts, 20.0, 2, 2, 100000)
    assert k_simple == len(ref20) and k_simple != k_pre
