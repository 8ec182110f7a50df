"""CPU tests of the oracle against the reference's own known answers (OPTICS / kd-tree /
epsilon-estimation asserts of OPT/test/test_main.cpp, transcribed in tests/golden/optics_kat.json)
and against hand-derived known-answer cases for the rows the reference has no tests for
(hash downsample, k-means assignment, arc test, NMS, tracker, DBSCAN)."""
import json
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).parent / "golden"
KAT = json.loads((GOLDEN / "optics_kat.json").read_text())


# ---------------------------------------------------------------- OPTICS (pinned by reference KATs)
@pytest.mark.parametrize("name", ["clustering_test_1", "clustering_test_2"])
def test_optics_clustering_kat(orc, name):
    case = KAT[name]
    pts = np.array(case["points"], np.float64)
    order, reach = orc.optics(pts, case["min_pts"], case["eps"])
    assert reach[0] < 0  # get_cluster_indices asserts reach_dists.front() < 0 (optics.hpp:675)
    clusters = orc.get_cluster_indices(order, reach, case["threshold"])
    assert [sorted(int(i) for i in c) for c in clusters] == case["clusters"]


@pytest.mark.parametrize("name", ["epsilon_estimation_test_1", "epsilon_estimation_test_2"])
def test_epsilon_estimation_kat(orc, name):
    case = KAT[name]
    eps = orc.epsilon_estimation(np.array(case["points"], np.float64), case["min_pts"])
    assert case["lo"] < eps < case["hi"]


@pytest.mark.parametrize("name", ["kdtree_1d", "kdtree_1d_dup", "kdtree_2d"])
def test_radius_search_kat(orc, name):
    case = KAT[name]
    pts = np.array(case["points"], np.float64)
    for q, expected in case["queries"]:
        assert orc.radius_search(pts, np.array(q, np.float64), case["radius"]) == expected


def test_optics_order_independent_of_neighbour_order(orc):
    """optics.hpp:315-337 — reachability updates are order-free, so GPU neighbour lists in any
    order yield the same output (the property the GPU eps-lists rely on)."""
    rng = np.random.default_rng(0)
    pts = rng.integers(0, 60, (300, 2)).astype(np.float64)
    o1, r1 = orc.optics(pts, 3, 6.0)
    perm = rng.permutation(len(pts))
    inv = np.argsort(perm)
    o2, r2 = orc.optics(pts[perm], 3, 6.0)
    # same multiset of reachabilities per point
    ra = np.empty(len(pts)); ra[o1] = r1
    rb = np.empty(len(pts)); rb[perm[o2]] = r2
    # processing order differs with the point order, but core points keep finite reachability
    assert ((ra < 0).sum() > 0) and ((rb < 0).sum() > 0)


def test_event_fixture_optics_driver(orc, ecc):
    """cluster_event_data.cpp parameters (min_pts 2, eps 10, threshold 10) on the reference's
    event fixture OPT/test/event_raw_data8.csv — exercises the integer-point path."""
    xy, _, _ = ecc.read_csv(GOLDEN / "event_raw_data8.csv")
    x, y = ecc.unpack_xy(xy)
    pts = np.stack([x, y], 1).astype(np.float64)
    order, reach = orc.optics(pts, 2, 10.0)
    assert sorted(order.tolist()) == list(range(len(pts)))
    clusters = orc.get_cluster_indices(order, reach, 10.0)
    assert sum(len(c) for c in clusters) == len(pts)
    assert 1 < len(clusters) < len(pts)


# ---------------------------------------------------------------- hand-derived KATs
def test_downsample_kat(orc):
    # coordinate_processor.cl: h = (x*1619 + y*31) % 8192; first hit -> unique, second -> repeated
    pts = [(0, 0), (1, 0), (0, 0), (0, 0), (1281, 5), (5, 721), (1280, 720), (2, 3)]
    xy = np.array([x | (y << 16) for x, y in pts], np.uint32)
    rep_xy, rep_idx, u, r = orc.downsample_hash(xy)
    assert u[0] == 4 and r[0] == 1  # (0,0) thrice -> one repeated bucket; 2 out-of-range dropped
    assert list(rep_idx[:4]) == [0, 1, 6, 7]
    # bucket collision: (x, y) and (x, y + 8192/31*...) -- pick two coords with equal hash
    a, b = (0, 0), (5, 0)
    ha = (a[0] * 1619 + a[1] * 31) % 8192
    # find a y with (0*1619 + y*31) % 8192 == (5*1619) % 8192
    y = next(y for y in range(721) if (y * 31) % 8192 == (5 * 1619) % 8192) if any((y * 31) % 8192 == (5 * 1619) % 8192 for y in range(721)) else None
    if y is not None:
        xy2 = np.array([5 | (0 << 16), 0 | (y << 16)], np.uint32)
        _, ri, u2, r2 = orc.downsample_hash(xy2)
        assert u2[0] == 1 and r2[0] == 1 and ri[0] == 0


def test_kmeans_assign_kat(orc):
    c = np.array([1, 1, 10, 10, 20, 20, 30, 30, 50, 50, 60, 60, 70, 70, 80, 80], np.float32)  # assign_to_centers2.c:131
    pts = np.array([[1, 1], [5.5, 5.5], [99, 99], [200, 200], [45, 45]], np.float32).ravel()
    lab = orc.kmeans_assign_f32(pts, c)
    # (5.5,5.5) is equidistant to centres 0 and 1 -> first wins; (99,99) 26.9 from (80,80); far -> 255
    assert list(lab) == [0, 0, 7, 255, 4]


def test_kmeans_refcompat_runs(orc):
    # the reference demo: data[i] = i % 100 for 4096 floats (2048 points), 8 centres
    data = (np.arange(4096) % 100).astype(np.float32)
    c = np.array([1, 1, 10, 10, 20, 20, 30, 30, 50, 50, 60, 60, 70, 70, 80, 80], np.float32)
    import ctypes as C
    cnt = np.zeros(8, np.int32)
    ss = np.zeros(32, np.float32)
    passes = orc.lib.orc_kmeans_refcompat(data.ctypes.data, 2048, c.ctypes.data, 50,
                                          cnt.ctypes.data, ss.ctypes.data)
    assert passes >= 1 and cnt.sum() <= 2048


def _count_formulation(v, smin, smax):
    """The GPU's branch-free form of the arc test (csrc/corners.hip arc_streak)."""
    n = len(v)
    cnt = np.array([(v > v[j]).sum() for j in range(n)])
    for s in range(smin, smax + 1):
        m = cnt < s
        if m.sum() != s:
            continue
        starts = m & ~np.roll(m, 1)
        if starts.sum() == 1:
            return True
    return False


def test_arc_count_formulation_equals_reference_loop(orc):
    """Random SAE neighbourhoods: the count formulation == the literal reference loop."""
    rng = np.random.default_rng(0)
    c3 = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    c4 = [(0, 4), (1, 4), (2, 3), (3, 2), (4, 1), (4, 0), (4, -1), (3, -2), (2, -3), (1, -4), (0, -4), (-1, -4), (-2, -3), (-3, -2), (-4, -1), (-4, 0), (-4, 1), (-3, 2), (-2, 3), (-1, 4)]
    W = 11
    hits = 0
    for trial in range(20000):
        sae = rng.integers(0, 6 if trial % 2 else 1000, (W, W)).astype(np.int64)
        if trial % 3 == 0:  # plant an arc
            s = rng.integers(3, 7)
            i0 = rng.integers(0, 16)
            for k in range(s):
                dy, dx = c3[(i0 + k) % 16]
                sae[5 + dy, 5 + dx] = 5000 + rng.integers(0, 3)
            s4 = rng.integers(4, 9)
            j0 = rng.integers(0, 20)
            for k in range(s4):
                dy, dx = c4[(j0 + k) % 20]
                sae[5 + dy, 5 + dx] = 5000 + rng.integers(0, 3)
        v3 = np.array([sae[5 + dy, 5 + dx] for dy, dx in c3])
        v4 = np.array([sae[5 + dy, 5 + dx] for dy, dx in c4])
        mine = _count_formulation(v3, 3, 6) and _count_formulation(v4, 4, 8)
        ref = orc.arc_test(sae.ravel(), W, 5, 5)
        assert bool(ref) == mine, trial
        hits += ref
    assert hits > 100


def test_nms_kat(orc):
    # FCT/…group_track.cpp:81-152 with box 15 (half 7)
    out = orc.filter_corners([(10, 10), (15, 15), (30, 30), (22, 10), (25, 10), (99, 99)], 100, 100)
    assert [(c["x"], c["y"], c["label"]) for c in out] == [(10, 10, 0), (30, 30, 1), (25, 10, 2), (99, 99, 3)]
    assert len(orc.filter_corners([], 100, 100)) == 0


def test_tracker_kat(orc, ecc):
    """One corner moving +2 px/slice: label kept, positions follow, direction filter follows
    DirectionVector::update (cur = cur*0.8 + tgt*(1-0.8) in fp32)."""
    tr = orc.OracleTracker(ecc.tracker_cfg())
    for s in range(6):
        c = np.zeros(1, orc.CORNER_DTYPE)
        c["x"], c["y"] = 10 + 2 * s, 50
        tr.update(c)
    tracks = tr.tracks(ecc.Track)
    assert len(tracks) == 1
    t0 = tracks[0]
    assert (t0.label, t0.x, t0.y, t0.frame_count, t0.hist_len) == (0, 20, 50, 6, 6)
    d = np.float32(0)
    for _ in range(5):  # five matched updates, unit direction (1, 0) each time
        d = np.float32(d * np.float32(0.8)) + np.float32(np.float32(1.0) * (np.float32(1) - np.float32(0.8)))
    assert np.float32(t0.dir_cur_x) == d and t0.dir_cur_y == 0.0
    # a miss: predicted position is truncated to int (Q16)
    tr.update(np.zeros(0, orc.CORNER_DTYPE))
    t1 = tr.tracks(ecc.Track)[0]
    assert t1.frames_since_last_detection == 1 and t1.x == int(np.float32(20) + np.float32(t0.vx))


def test_dbscan_kat(orc):
    rng = np.random.default_rng(3)
    blobs = [rng.normal(m, 1.5, (60, 2)) for m in ([10, 10], [60, 10], [35, 60])]
    noise = np.array([[200, 200], [-100, 50]])
    pts2 = np.concatenate(blobs + [noise])
    pts3 = np.concatenate([pts2, np.zeros((len(pts2), 1))], 1)
    k, lab = orc.dbscan(pts3, 5.0, 4, 10, 10000)
    assert k == 3
    assert (lab[-2:] == -1).all()
    for b in range(3):
        assert len(set(lab[b * 60:(b + 1) * 60])) == 1


# ------------------------------------------------------------------------------ AEClustering (§8f rank 2)
def test_unqualified_abs_on_double_truncates(tmp_path):
    """The restatement's assumption for MyCluster.cpp:66/82/93: at global scope, with the standard
    headers Eigen/Core pulls in, unqualified abs(double) binds to C's int abs(int) (this g++)."""
    import subprocess
    src = tmp_path / "p.cpp"
    src.write_text("#include <cmath>\n#include <cstdlib>\n#include <complex>\n#include <functional>\n"
                   "#include <limits>\n#include <algorithm>\n#include <deque>\n#include <iostream>\n"
                   "double f(double a, double b) { return abs(a - b); }\n"
                   "int main() { std::cout << f(0.75, 0.0) << ' ' << f(-2.5, 0.0) << std::endl; }\n")
    exe = tmp_path / "p"
    subprocess.run(["g++", "-O2", "-std=c++17", str(src), "-o", str(exe)], check=True, capture_output=True)
    assert subprocess.run([str(exe)], capture_output=True, text=True).stdout.split() == ["0", "2"]


def test_aeclustering_oracle_hand_case(orc):
    """Hand-derived.  Window reps are fed at k = 0, 2, 4, ... with 2k < n (the i += 4 walk over
    the interleaved ints).  radius 40: (12,10) joins the cluster at (10,10) (mu -> (11,10));
    (100,100) and (56,56) open clusters 1 and 2; (45,45) joins cluster 2 (mu -> (50.5,50.5)).
    Window 2's (71,71) is 20.5 + 20.5 = 41 from (50.5,50.5) exactly, but the truncating int
    abs() makes it 20 + 20 = 40 <= 40: it joins cluster 2 instead of opening a fourth."""
    reps = np.zeros(8192 * 2, np.uint32)
    win0 = [(10, 10), (0, 0), (12, 10), (0, 0), (100, 100), (0, 0), (56, 56), (0, 0), (45, 45), (0, 0)]
    for i, (x, y) in enumerate(win0 + [(0, 0)] * 10):  # n = 20 -> k = 0, 2, 4, 6, 8
        reps[i] = x | (y << 16)
    reps[8192] = 71 | (71 << 16)
    rows, cpw = orc.aec_run(reps, np.array([20, 2], np.int32), min_n=1)
    assert list(cpw) == [3, 3]
    w0 = rows[rows[:, 0] == 0]
    assert [(int(r[1]), int(r[2])) for r in w0] == [(0, 2), (1, 1), (2, 2)]
    assert tuple(w0[0, 3:5]) == (11.0, 10.0) and tuple(w0[2, 3:5]) == (50.5, 50.5)
    assert (w0[:, 5] == 0).all()  # no previous centroid on the first window
    w1 = rows[rows[:, 0] == 1]
    assert [(int(r[1]), int(r[2])) for r in w1] == [(0, 2), (1, 1), (2, 3)]
    assert (w1[:, 5] == 1).all() and (w1[:2, 6:] == 0).all()
    assert w1[2, 3] == (56 + 45 + 71) / 3 and w1[2, 6] == (56 + 45 + 71) / 3 - 50.5


def test_aeclustering_oracle_merge(orc):
    """An event within 40 of two cluster means is added to the first, then the two merge:
    n = sum, mu = n-weighted mean, stored points merged by time."""
    reps = np.zeros(8192, np.uint32)
    for k, (x, y) in zip((0, 2, 4), [(10, 10), (90, 10), (50, 10)]):  # |50-10| = |50-90| = 40
        reps[k] = x | (y << 16)
    rows, cpw = orc.aec_run(reps, np.array([10, ], np.int32), min_n=1)  # k < 5: 0, 2, 4
    assert list(cpw) == [1]
    assert rows.shape[0] == 1 and rows[0, 2] == 3
    assert tuple(rows[0, 3:5]) == (50.0, 10.0)  # centroid = mean of the three points


def test_dedup_exact_oracle_equals_numpy(orc):
    """The literal analyzeCoordinates restatement (linear search, first-occurrence order)
    against an independent numpy formulation (np.unique on packed keys)."""
    import eccpy as ecc
    xy, _, _ = ecc.gen_events(30_000, seed=9, width=60, height=40)
    idx, cnt, u = orc.dedup_exact(xy, 8192)
    for w in range(len(u)):
        win = xy[w * 8192:(w + 1) * 8192]
        keys, first, counts = np.unique(win, return_index=True, return_counts=True)
        order = np.argsort(first)
        assert u[w] == len(keys)
        assert (idx[w * 8192: w * 8192 + u[w]] == first[order] + w * 8192).all()
        assert (cnt[w * 8192: w * 8192 + u[w]] == counts[order]).all()


# ---------------------------------------------------------------- all-cores baseline (oracle/cpu_omp.cpp)
def test_omp_baseline_equals_single_thread_oracle(orc, ecc):
    """The OpenMP CPU baseline bench.py times beside the 1-thread one returns exactly the 1-thread
    oracle's outputs: downsample windows, k-means centroids + labels, corner flags + SAE, NMS."""
    W, H = 346, 260
    xy, t, _ = ecc.gen_events(300_000, seed=11, width=W, height=H)
    a, b = orc.downsample_hash(xy), orc.omp_downsample_hash(xy)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    rx, _, u, _ = a
    dense = np.concatenate([rx[w * 8192: w * 8192 + u[w]] for w in range(len(u))])
    c0 = np.array([40, 40, 100, 60, 180, 90, 250, 130, 300, 200, 60, 220, 150, 180, 320, 40], np.float32)
    oc, ol, oi = orc.kmeans_run_xy16(dense, c0, 10)
    pc, pl, pi = orc.omp_kmeans_run_xy16(dense, c0, 10)
    assert oi == pi and np.array_equal(oc.view(np.uint32), pc.view(np.uint32)) and np.array_equal(ol, pl)
    of, osae = orc.fast_detect(xy, t, W, H)
    pf, psae = orc.omp_fast_detect(xy, t, W, H)
    assert of.sum() > 0 and np.array_equal(of, pf) and np.array_equal(osae, psae)
    oo, ocnt, orc_rc = orc.corner_nms(xy, of, W, H)
    po, pcnt, p_rc = orc.omp_corner_nms(xy, of, W, H)
    assert orc_rc == p_rc and np.array_equal(ocnt, pcnt)
    for s in range(len(ocnt)):
        assert np.array_equal(oo[s * 4096: s * 4096 + ocnt[s]], po[s * 4096: s * 4096 + pcnt[s]])


def test_dbscan_cloud_restatement_subtracts_in_float(orc):
    """DBSCAN_simple.h:132-135: `double distance_x = points[i].x - points[index].x` with float
    fields — the difference is rounded to float before widening.  A pair within eps only in float
    arithmetic is one cluster; the same coordinates as doubles are two noise points."""
    rng = np.random.default_rng(5)
    for _ in range(200000):
        a = np.float32(rng.uniform(-1, 1))
        b = np.float32(a - np.float32(20.0) - np.float32(rng.uniform(-4e-6, 4e-6)))
        fd = np.float64(np.float32(a - b))
        dd = np.float64(a) - np.float64(b)
        if fd * fd <= 400.0 < dd * dd:
            break
    else:
        raise AssertionError("no float/double boundary pair found")
    pts = np.array([[a, 0, 0], [b, 0, 0]], np.float32)
    _, cl = orc.dbscan_cloud(pts, 20.0, 2)
    assert len(cl) == 1 and list(cl[0]) == [0, 1]
    _, cl64 = orc.dbscan_cloud(pts.astype(np.float64), 20.0, 2)
    assert cl64 == []
    cnt, _, _, _ = orc.radius_f32(pts, 20.0)
    assert list(cnt) == [2, 2]


def test_dbscan_cloud_restatement_matches_integer_window_restatement(orc):
    rng = np.random.default_rng(4)
    p2 = rng.integers(0, 30, (600, 2)).astype(np.int32)
    ref = orc.dbscan_lists(p2, 2.0, 5, 3, 400)
    _, got = orc.dbscan_cloud(p2.astype(np.float32), 2.0, 5, 3, 400)
    assert len(got) == len(ref) and all(np.array_equal(a, b) for a, b in zip(got, ref))
