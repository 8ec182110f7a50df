"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference algorithms (oracle/oracle.cpp).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / the CPU baseline.  It never backs a product code path.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "liboracle.so"


def build() -> None:
    import subprocess
    subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True, stdout=subprocess.DEVNULL)


if not LIB_PATH.exists():
    build()
lib = C.CDLL(str(LIB_PATH))

P = C.c_void_p
i64, i32, f32, f64 = C.c_int64, C.c_int32, C.c_float, C.c_double
_sigs = {
    "orc_downsample_hash": (C.c_int, [P, i64, i32, i32, i32, i32, i32, i32, P, P, P, P]),
    "orc_dedup_exact": (C.c_int, [P, i64, i32, P, P, P]),
    "orc_kmeans_assign_f32": (C.c_int, [P, i64, P, i32, f32, P]),
    "orc_kmeans_run_f32": (C.c_int, [P, i64, P, i32, i32, f32, f32, P, P]),
    "orc_kmeans_run_xy16": (C.c_int, [P, i64, P, i32, i32, f32, f32, P, P]),
    "orc_kmeans_refcompat": (C.c_int, [P, i64, P, i32, P, P]),
    "orc_kmeans_refcompat_pass": (C.c_int, [P, i64, P, P, P, P]),
    "orc_arc_test": (C.c_int, [P, i32, i32, i32]),
    "orc_fast_detect": (C.c_int, [P, P, i64, i32, i32, i32, i32, i32, i32, P, P]),
    "orc_filter_corners": (C.c_int, [P, i32, i32, i32, i32, P, i32]),
    "orc_corner_nms": (C.c_int, [P, P, i64, i32, i32, i32, i32, i32, P, P]),
    "orc_tracker_create": (P, [P]),
    "orc_tracker_destroy": (None, [P]),
    "orc_tracker_update": (C.c_int, [P, P, i32]),
    "orc_tracker_get_tracks": (C.c_int, [P, P, i32]),
    "orc_tracker_get_groups": (C.c_int, [P, P, i32, P, i32]),
    "orc_eps_neighbours": (C.c_int, [P, i64, i64, P, f64, i32, P, P, P, P, i64]),
    "orc_dbscan": (C.c_int, [P, i32, f64, i32, i32, i32, P]),
    "orc_epsilon_estimation": (f64, [P, i32, i32, i32]),
    "orc_optics": (C.c_int, [P, i32, i32, i32, f64, P, P]),
    "orc_get_cluster_indices": (C.c_int, [P, i32, f64, P]),
    "orc_radius_search": (C.c_int, [P, i32, i32, P, f64, P, i32]),
    "orc_kmeans_partial_xy16": (C.c_int, [P, i64, P, i32, f32, P]),
    "orc_evt2_decode": (i64, [P, i64, P, P, P, i64]),
    "orc_evt3_decode": (i64, [P, i64, P, P, P, i64]),
    "orc_evt2_encode": (i64, [P, P, P, i64, C.c_uint64, i32, P, i64]),
    "orc_evt3_encode": (i64, [P, P, P, i64, C.c_uint64, i32, i32, P, i64]),
    "orc_reslice_n_us": (i64, [P, i64, i64, P, i64]),
    "orc_dbscan_lists": (C.c_int, [P, i32, f64, i32, i32, i32, P, P, i64]),
    "orc_dbscan_cloud_f32": (C.c_int, [P, i32, i32, f64, i32, i32, i32, P, P, P, i64]),
    "orc_dbscan_cloud_f64": (C.c_int, [P, i32, i32, f64, i32, i32, i32, P, P, P, i64]),
    "orc_radius_f32": (C.c_int, [P, i32, i32, f64, i32, P, P, P, P, i64]),
    "orc_aec_run": (i64, [P, P, i64, i64, i32, f64, i32, f64, i32, P, i64, P]),
}
for _n, (_r, _a) in _sigs.items():
    f = getattr(lib, _n)
    f.restype = _r
    f.argtypes = _a


def _p(a):
    return None if a is None else a.ctypes.data


def downsample_hash(xy, window=8192, x_max=1280, y_max=720, mult_x=1619, mult_y=31, nb=8192):
    xy = np.ascontiguousarray(xy, np.uint32)
    n = len(xy)
    nw = (n + window - 1) // window
    rep_xy = np.zeros(nw * window, np.uint32)
    rep_idx = np.zeros(nw * window, np.uint32)
    u = np.zeros(nw, np.int32)
    r = np.zeros(nw, np.int32)
    rc = lib.orc_downsample_hash(_p(xy), n, window, x_max, y_max, mult_x, mult_y, nb, _p(rep_xy),
                                 _p(rep_idx), _p(u), _p(r))
    assert rc == 0
    return rep_xy, rep_idx, u, r


def dedup_exact(xy, window=8192):
    """analyzeCoordinates per window: (uniq_idx, uniq_cnt, n_unique), padded per window."""
    xy = np.ascontiguousarray(xy, np.uint32)
    n = len(xy)
    nw = (n + window - 1) // window
    idx = np.zeros(nw * window, np.uint32)
    cnt = np.zeros(nw * window, np.int32)
    u = np.zeros(nw, np.int32)
    assert lib.orc_dedup_exact(_p(xy), n, window, _p(idx), _p(cnt), _p(u)) == 0
    return idx, cnt, u


def kmeans_assign_f32(xy2, centroids, thr=50.0):
    xy2 = np.ascontiguousarray(xy2, np.float32)
    c = np.ascontiguousarray(centroids, np.float32)
    n = xy2.size // 2
    lab = np.zeros(n, np.uint8)
    lib.orc_kmeans_assign_f32(_p(xy2), n, _p(c), c.size // 2, thr, _p(lab))
    return lab


def kmeans_run_xy16(xy, centroids, max_iters, thr=50.0, tol=-1.0):
    xy = np.ascontiguousarray(xy, np.uint32)
    c = np.array(centroids, np.float32).copy()
    lab = np.zeros(len(xy), np.uint8)
    it = np.zeros(1, np.int32)
    lib.orc_kmeans_run_xy16(_p(xy), len(xy), _p(c), c.size // 2, max_iters, thr, tol, _p(lab), _p(it))
    return c, lab, int(it[0])


def kmeans_run_f32(xy2, centroids, max_iters, thr=50.0, tol=-1.0):
    xy2 = np.ascontiguousarray(xy2, np.float32)
    c = np.array(centroids, np.float32).copy()
    n = xy2.size // 2
    lab = np.zeros(n, np.uint8)
    it = np.zeros(1, np.int32)
    lib.orc_kmeans_run_f32(_p(xy2), n, _p(c), c.size // 2, max_iters, thr, tol, _p(lab), _p(it))
    return c, lab, int(it[0])


def fast_detect(xy, t, W, H, slice_events=16384, margin=4, border_mode=0, first_detect=1, sae=None):
    xy = np.ascontiguousarray(xy, np.uint32)
    t = np.ascontiguousarray(t, np.int64)
    sae = np.zeros(W * H, np.int64) if sae is None else np.array(sae, np.int64).copy()
    flags = np.zeros(len(xy), np.uint8)
    rc = lib.orc_fast_detect(_p(xy), _p(t), len(xy), W, H, slice_events, margin, border_mode,
                             first_detect, _p(sae), _p(flags))
    assert rc == 0
    return flags, sae


def arc_test(sae, W, x, y):
    sae = np.ascontiguousarray(sae, np.int64)
    return lib.orc_arc_test(_p(sae), W, x, y)


CORNER_DTYPE = np.dtype([("x", np.int32), ("y", np.int32), ("label", np.int32)])


def filter_corners(corners_xy, W, H, box=15):
    c = np.zeros(len(corners_xy), CORNER_DTYPE)
    if len(corners_xy):
        c["x"] = [p[0] for p in corners_xy]
        c["y"] = [p[1] for p in corners_xy]
    out = np.zeros(max(len(corners_xy), 1), CORNER_DTYPE)
    k = lib.orc_filter_corners(_p(c), len(c), W, H, box, _p(out), len(out))
    return out[:k]


def corner_nms(xy, flags, W, H, slice_events=16384, box=15, cap=4096):
    xy = np.ascontiguousarray(xy, np.uint32)
    flags = np.ascontiguousarray(flags, np.uint8)
    ns = (len(xy) + slice_events - 1) // slice_events
    out = np.zeros(ns * cap, CORNER_DTYPE)
    counts = np.zeros(ns, np.int32)
    rc = lib.orc_corner_nms(_p(xy), _p(flags), len(xy), slice_events, W, H, box, cap, _p(out), _p(counts))
    return out, counts, rc


class OracleTracker:
    def __init__(self, cfg):
        self.h = lib.orc_tracker_create(C.byref(cfg))

    def update(self, corners: np.ndarray):
        corners = np.ascontiguousarray(corners, CORNER_DTYPE)
        lib.orc_tracker_update(self.h, _p(corners), len(corners))

    def tracks(self, track_type, cap=65536):
        buf = (track_type * cap)()
        n = lib.orc_tracker_get_tracks(self.h, buf, cap)
        return [buf[i] for i in range(min(n, cap))]

    def groups(self, group_type, cap=65536):
        buf = (group_type * cap)()
        labels = np.zeros(cap, np.int32)
        n = lib.orc_tracker_get_groups(self.h, buf, cap, _p(labels), cap)
        return [buf[i] for i in range(min(n, cap))], labels

    def __del__(self):
        try:
            lib.orc_tracker_destroy(self.h)
        except Exception:
            pass


def eps_neighbours(xy, n_segs, stride, seg_counts, eps, min_pts, want_lists=True):
    xy = np.ascontiguousarray(xy, np.uint32)
    total = n_segs * stride
    counts = np.zeros(total, np.int32)
    core = np.zeros(total, np.float64)
    offsets = np.zeros(total + 1, np.int64)
    sc = None if seg_counts is None else np.ascontiguousarray(seg_counts, np.int32)
    # first pass for the list size
    lib.orc_eps_neighbours(_p(xy), n_segs, stride, _p(sc), eps, min_pts, _p(counts), _p(core),
                           _p(offsets), None, 0)
    nbr = None
    if want_lists:
        nbr = np.zeros(max(int(offsets[-1]), 1), np.int32)
        lib.orc_eps_neighbours(_p(xy), n_segs, stride, _p(sc), eps, min_pts, None, None,
                               _p(offsets), _p(nbr), len(nbr))
    return counts, core, offsets, nbr


def dbscan(pts3, eps, min_pts, min_size=1, max_size=2**31 - 1):
    pts3 = np.ascontiguousarray(pts3, np.float32)
    n = pts3.shape[0]
    lab = np.zeros(n, np.int32)
    k = lib.orc_dbscan(_p(pts3), n, eps, min_pts, min_size, max_size, _p(lab))
    return k, lab


def dbscan_cloud(pts, eps, min_pts, min_size=1, max_size=2**31 - 1):
    """DBSCAN_simple.h:27-142 literally over an (n, dim) float32 or float64 cloud: (labels, clusters)
    with clusters a list of sorted index arrays in output order."""
    pts = np.ascontiguousarray(pts)
    assert pts.dtype in (np.float32, np.float64) and pts.ndim == 2
    n, dim = pts.shape
    fn = lib.orc_dbscan_cloud_f32 if pts.dtype == np.float32 else lib.orc_dbscan_cloud_f64
    lab = np.zeros(n, np.int32)
    cap = max(1, 2 * n)
    while True:
        offs = np.zeros(n + 2, np.int64)
        mem = np.empty(cap, np.int32)
        nc = fn(_p(pts), n, dim, eps, min_pts, min_size, max_size, _p(lab), _p(offs), _p(mem), cap)
        if offs[nc] <= cap:
            return lab, [mem[offs[c]:offs[c + 1]].copy() for c in range(nc)]
        cap = int(offs[nc])


def radius_f32(pts, eps, min_pts=1, want_lists=True):
    """Brute-force eps-balls of an (n, dim) float32 cloud with float per-axis differences:
    (counts, core distances, offsets, ascending neighbour lists)."""
    pts = np.ascontiguousarray(pts, np.float32)
    n, dim = pts.shape
    counts = np.zeros(n, np.int32)
    core = np.zeros(n, np.float64)
    offs = np.zeros(n + 1, np.int64)
    lib.orc_radius_f32(_p(pts), n, dim, eps, min_pts, _p(counts), _p(core), _p(offs), None, 0)
    nbr = None
    if want_lists:
        nbr = np.zeros(max(int(offs[-1]), 1), np.int32)
        lib.orc_radius_f32(_p(pts), n, dim, eps, min_pts, None, None, _p(offs), _p(nbr), len(nbr))
    return counts, core, offs, nbr


def epsilon_estimation(pts, min_pts):
    pts = np.ascontiguousarray(pts, np.float64)
    n, d = pts.shape
    return lib.orc_epsilon_estimation(_p(pts), n, d, min_pts)


def optics(pts, min_pts, eps=-1.0):
    pts = np.ascontiguousarray(pts, np.float64)
    n, d = pts.shape
    order = np.zeros(n, np.int64)
    reach = np.zeros(n, np.float64)
    lib.orc_optics(_p(pts), n, d, min_pts, eps, _p(order), _p(reach))
    return order, reach


def get_cluster_indices(order, reach, thr):
    reach = np.ascontiguousarray(reach, np.float64)
    cl = np.zeros(len(reach), np.int32)
    k = lib.orc_get_cluster_indices(_p(reach), len(reach), thr, _p(cl))
    return [list(np.asarray(order)[cl == c]) for c in range(k)]


def radius_search(pts, q, r):
    pts = np.ascontiguousarray(pts, np.float64)
    q = np.ascontiguousarray(q, np.float64)
    n, d = pts.shape
    out = np.zeros(n, np.int64)
    k = lib.orc_radius_search(_p(pts), n, d, _p(q), r, _p(out), n)
    return list(out[:k])


def kmeans_partial_xy16(xy, centroids, thr=50.0):
    xy = np.ascontiguousarray(xy, np.uint32)
    c = np.ascontiguousarray(centroids, np.float32)
    acc = np.zeros(3 * (c.size // 2), np.int64)
    lib.orc_kmeans_partial_xy16(_p(xy), len(xy), _p(c), c.size // 2, thr, _p(acc))
    return acc


# ---- RAW ingest (EVT 2.0 / 3.0) --------------------------------------------------------------
def evt_encode(fmt, xy, t, p, seed=1, noise_pct=5, vect_pct=70):
    """Encodes events into an EVT 2.0 (u32) or EVT 3.0 (u16) word stream."""
    xy = np.ascontiguousarray(xy, np.uint32)
    t = np.ascontiguousarray(t, np.int64)
    p = np.ascontiguousarray(p, np.uint8)
    n = len(xy)
    if fmt == 2:
        cap = 4 * n + 16
        out = np.empty(cap, np.uint32)
        k = lib.orc_evt2_encode(_p(xy), _p(t), _p(p), n, seed, noise_pct, _p(out), cap)
    else:
        cap = 8 * n + 64 + 2 * int((t[-1] >> 24) + 1 if n else 0)
        out = np.empty(cap, np.uint16)
        k = lib.orc_evt3_encode(_p(xy), _p(t), _p(p), n, seed, noise_pct, vect_pct, _p(out), cap)
    assert k <= cap
    return out[:k].copy()


def evt_decode(fmt, words):
    words = np.ascontiguousarray(words, np.uint32 if fmt == 2 else np.uint16)
    n = len(words)
    cap = n * (1 if fmt == 2 else 12)
    xy = np.empty(cap, np.uint32)
    t = np.empty(cap, np.int64)
    p = np.empty(cap, np.uint8)
    fn = lib.orc_evt2_decode if fmt == 2 else lib.orc_evt3_decode
    k = fn(_p(words), n, _p(xy), _p(t), _p(p), cap)
    return xy[:k].copy(), t[:k].copy(), p[:k].copy()


def reslice_n_us(t, period, max_slices=None):
    t = np.ascontiguousarray(t, np.int64)
    if max_slices is None:
        max_slices = 1 if len(t) == 0 else int((t[-1] - (t[0] // period) * period) // period + 1)
    bounds = np.zeros(max_slices + 1, np.int64)
    ns = lib.orc_reslice_n_us(_p(t), len(t), period, _p(bounds), max_slices)
    return bounds, int(ns)


def dbscan_lists(pts_xy, eps, min_pts, min_size=1, max_size=1 << 30):
    """Reference DBSCAN output (DBSCAN_simple.h:27-90) as a list of sorted index arrays."""
    pts = np.ascontiguousarray(np.asarray(pts_xy, np.int32).reshape(-1, 2))
    n = len(pts)
    cap = max(1, 4 * n)
    while True:
        offs = np.zeros(n + 2, np.int64)
        mem = np.empty(cap, np.int32)
        nc = lib.orc_dbscan_lists(_p(pts), n, eps, min_pts, min_size, max_size, _p(offs), _p(mem), cap)
        if offs[nc] <= cap:
            return [mem[offs[c]:offs[c + 1]].copy() for c in range(nc)]
        cap = int(offs[nc])


def aec_run(rep_xy, win_unique, stride=8192, sz_buffer=800, radius=40.0, kappa=0, alpha=0.5, min_n=10):
    """AEClustering over the downsample windows (DSA slice path) -> (rows[k, 8], clusters per window);
    row = window, cluster id, n, centroid x, y, has_prev, flow dx, dy."""
    rep_xy = np.ascontiguousarray(rep_xy, np.uint32)
    u = np.ascontiguousarray(win_unique, np.int32)
    nw = len(u)
    cap = 1 << 16
    while True:
        rows = np.zeros((cap, 8), np.float64)
        cpw = np.zeros(max(nw, 1), np.int32)
        k = lib.orc_aec_run(_p(rep_xy), _p(u), nw, stride, sz_buffer, radius, kappa, alpha, min_n, _p(rows), cap,
                            _p(cpw))
        if k <= cap:
            return rows[:k].copy(), cpw[:nw].copy()
        cap = int(k)


# ------------------------------------------------------------------------------------------
# All-cores CPU baseline (oracle/cpu_omp.cpp, OpenMP): the same restatement with its parallel
# stages spread over the host's threads (OMP_NUM_THREADS).  Same outputs as the functions above.
# ------------------------------------------------------------------------------------------
OMP_LIB_PATH = ORACLE_DIR / "libcpu_omp.so"
_omp = None


def omp_lib():
    global _omp
    if _omp is None:
        if not OMP_LIB_PATH.exists():
            build()
        _omp = C.CDLL(str(OMP_LIB_PATH))
        for _n, (_r, _a) in {
            "omp_threads": (C.c_int, []),
            "omp_downsample_hash": _sigs["orc_downsample_hash"],
            "omp_kmeans_run_xy16": _sigs["orc_kmeans_run_xy16"],
            "omp_fast_detect": _sigs["orc_fast_detect"],
            "omp_corner_nms": _sigs["orc_corner_nms"],
        }.items():
            f = getattr(_omp, _n)
            f.restype = _r
            f.argtypes = _a
    return _omp


def omp_threads():
    return omp_lib().omp_threads()


def omp_downsample_hash(xy, window=8192, x_max=1280, y_max=720, mult_x=1619, mult_y=31, nb=8192):
    xy = np.ascontiguousarray(xy, np.uint32)
    n = len(xy)
    nw = (n + window - 1) // window
    rep_xy = np.zeros(nw * window, np.uint32)
    rep_idx = np.zeros(nw * window, np.uint32)
    u = np.zeros(nw, np.int32)
    r = np.zeros(nw, np.int32)
    rc = omp_lib().omp_downsample_hash(_p(xy), n, window, x_max, y_max, mult_x, mult_y, nb, _p(rep_xy),
                                       _p(rep_idx), _p(u), _p(r))
    assert rc == 0
    return rep_xy, rep_idx, u, r


def omp_kmeans_run_xy16(xy, centroids, max_iters, thr=50.0, tol=-1.0):
    xy = np.ascontiguousarray(xy, np.uint32)
    c = np.array(centroids, np.float32).copy()
    lab = np.zeros(len(xy), np.uint8)
    it = np.zeros(1, np.int32)
    omp_lib().omp_kmeans_run_xy16(_p(xy), len(xy), _p(c), c.size // 2, max_iters, thr, tol, _p(lab), _p(it))
    return c, lab, int(it[0])


def omp_fast_detect(xy, t, W, H, slice_events=16384, margin=4, border_mode=0, first_detect=1):
    xy = np.ascontiguousarray(xy, np.uint32)
    t = np.ascontiguousarray(t, np.int64)
    sae = np.zeros(W * H, np.int64)
    flags = np.zeros(len(xy), np.uint8)
    rc = omp_lib().omp_fast_detect(_p(xy), _p(t), len(xy), W, H, slice_events, margin, border_mode,
                                   first_detect, _p(sae), _p(flags))
    assert rc == 0
    return flags, sae


def omp_corner_nms(xy, flags, W, H, slice_events=16384, box=15, cap=4096):
    xy = np.ascontiguousarray(xy, np.uint32)
    flags = np.ascontiguousarray(flags, np.uint8)
    ns = (len(xy) + slice_events - 1) // slice_events
    out = np.zeros(ns * cap, CORNER_DTYPE)
    counts = np.zeros(ns, np.int32)
    rc = omp_lib().omp_corner_nms(_p(xy), _p(flags), len(xy), slice_events, W, H, box, cap, _p(out), _p(counts))
    return out, counts, rc
