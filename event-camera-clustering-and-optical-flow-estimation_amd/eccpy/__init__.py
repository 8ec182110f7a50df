"""ctypes binding of libecc (the MI355X-native event-camera clustering / corner pipeline).

Thin Python mirror of the C ABI in include/ecc.h, used by tests/ and bench.py.  The product
path is the HIP library: importing this module fails loudly when lib/libecc.so is missing, and
every compute call goes through the C ABI (no CPU fallback exists here).
"""
from __future__ import annotations

import ctypes as C
import json
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent.parent
LIB_PATH = Path(os.environ.get("ECC_LIB", PKG_DIR / "lib" / "libecc.so"))

if not LIB_PATH.exists():
    raise ImportError(f"libecc not built: {LIB_PATH} missing (run `make -C {PKG_DIR}` or "
                      f"__graft_entry__.build())")
lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)

OK, ERR_INVALID, ERR_HIP, ERR_UNSORTED_TIME, ERR_CAPACITY, ERR_NOMEM, ERR_NO_DEVICE = 0, -1, -2, -3, -4, -5, -6
TRACK_HIST_MAX = 16


class EccError(RuntimeError):
    def __init__(self, rc: int, what: str = ""):
        msg = lib.ecc_status_string(rc).decode()
        super().__init__(f"{what}: {msg} ({rc})" if what else f"{msg} ({rc})")
        self.rc = rc


def check(rc: int, what: str = "") -> int:
    if rc != OK:
        raise EccError(rc, what)
    return rc


# ---------------------------------------------------------------- structs (match include/ecc.h)
class HashCfg(C.Structure):
    _fields_ = [("window", C.c_int32), ("x_max", C.c_int32), ("y_max", C.c_int32),
                ("mult_x", C.c_int32), ("mult_y", C.c_int32), ("n_buckets", C.c_int32)]


class KmeansCfg(C.Structure):
    _fields_ = [("k", C.c_int32), ("max_iters", C.c_int32), ("threshold", C.c_float),
                ("tol", C.c_float)]


class CornerCfg(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("slice_events", C.c_int32),
                ("margin", C.c_int32), ("border_mode", C.c_int32),
                ("first_detect_slice", C.c_int32), ("any_order", C.c_int32)]


class RawInfo(C.Structure):
    _fields_ = [("format", C.c_int32), ("width", C.c_int32), ("height", C.c_int32),
                ("word_bytes", C.c_int32), ("header_bytes", C.c_int64), ("n_words", C.c_int64)]


class Corner(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("label", C.c_int32)]


CORNER_DTYPE = np.dtype([("x", np.int32), ("y", np.int32), ("label", np.int32)])


class TrackerCfg(C.Structure):
    _fields_ = [("max_distance", C.c_float), ("max_frames", C.c_int32),
                ("history_size", C.c_int32), ("frames_to_skip", C.c_int32),
                ("damping", C.c_float), ("smoothing", C.c_float), ("group_radius", C.c_float)]


class Track(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("label", C.c_int32),
                ("frame_count", C.c_int32), ("is_matched", C.c_int32),
                ("frames_since_last_detection", C.c_int32), ("hist_len", C.c_int32),
                ("hist_x", C.c_int32 * TRACK_HIST_MAX), ("hist_y", C.c_int32 * TRACK_HIST_MAX),
                ("vx", C.c_float), ("vy", C.c_float), ("dir_cur_x", C.c_float),
                ("dir_cur_y", C.c_float), ("dir_tgt_x", C.c_float), ("dir_tgt_y", C.c_float),
                ("group_id", C.c_int32)]


class Group(C.Structure):
    _fields_ = [("id", C.c_int32), ("n_labels", C.c_int32), ("first_label_offset", C.c_int32),
                ("avg_vx", C.c_float), ("avg_vy", C.c_float), ("cx", C.c_float),
                ("cy", C.c_float), ("radius", C.c_float)]


class GenCfg(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("width", C.c_int32), ("height", C.c_int32),
                ("rate_mev_s", C.c_double), ("t0", C.c_int64), ("n_polygons", C.c_int32),
                ("n_blobs", C.c_int32), ("frac_edges", C.c_float), ("frac_blobs", C.c_float)]


P = C.c_void_p
i64 = C.c_int64
i32 = C.c_int32
_sigs = {
    "ecc_version": (C.c_int, []),
    "ecc_status_string": (C.c_char_p, [C.c_int]),
    "ecc_ctx_create": (C.c_int, [C.POINTER(P), C.c_int]),
    "ecc_ctx_destroy": (C.c_int, [P]),
    "ecc_ctx_last_error": (C.c_char_p, [P]),
    "ecc_stream_sync": (C.c_int, [P]),
    "ecc_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "ecc_set_device": (C.c_int, [C.c_int]),
    "ecc_dev_alloc": (C.c_int, [C.POINTER(P), C.c_size_t]),
    "ecc_dev_free": (C.c_int, [P]),
    "ecc_memset_async": (C.c_int, [P, C.c_int, C.c_size_t, P]),
    "ecc_memcpy_h2d": (C.c_int, [P, P, C.c_size_t, P]),
    "ecc_memcpy_d2h": (C.c_int, [P, P, C.c_size_t, P]),
    "ecc_memcpy_d2d": (C.c_int, [P, P, C.c_size_t, P]),
    "ecc_stream_create": (C.c_int, [C.POINTER(P)]),
    "ecc_stream_destroy": (C.c_int, [P]),
    "ecc_event_create": (C.c_int, [C.POINTER(P)]),
    "ecc_event_destroy": (C.c_int, [P]),
    "ecc_event_record": (C.c_int, [P, P]),
    "ecc_event_elapsed_ms": (C.c_int, [C.POINTER(C.c_float), P, P]),
    "ecc_stream_wait_event": (C.c_int, [P, P]),
    "ecc_ctx_set_timing": (C.c_int, [P, C.c_int]),
    "ecc_ctx_timing_reset": (C.c_int, [P]),
    "ecc_ctx_timing_report": (C.c_int, [P, C.c_char_p, C.c_size_t]),
    "ecc_util_sqrt_f32": (C.c_int, [P, P, P, i64, P]),
    "ecc_graph_begin": (C.c_int, [P]),
    "ecc_graph_end": (C.c_int, [P, C.POINTER(P)]),
    "ecc_graph_launch": (C.c_int, [P, P]),
    "ecc_graph_destroy": (C.c_int, [P]),
    "ecc_hash_cfg_default": (None, [C.POINTER(HashCfg)]),
    "ecc_dedup_exact": (C.c_int, [P, P, i64, i32, P, P, P, P]),
    "ecc_downsample_hash": (C.c_int, [P, P, i64, C.POINTER(HashCfg), P, P, P, P, P]),
    "ecc_kmeans_cfg_default": (None, [C.POINTER(KmeansCfg)]),
    "ecc_kmeans_run_xy16": (C.c_int, [P, P, i64, i64, P, C.POINTER(KmeansCfg), P, P, P, P]),
    "ecc_kmeans_run_f32": (C.c_int, [P, P, i64, C.POINTER(KmeansCfg), P, P, P, P]),
    "ecc_kmeans_run_xy16_frame": (C.c_int, [P, P, i64, i64, P, i32, i32, C.POINTER(KmeansCfg), P, P, P, P]),
    "ecc_kmeans_refcompat_f32": (C.c_int, [P, P, i64, P, i32, P, P, P, P]),
    "ecc_kmeans_run_f32_engine": (C.c_int, [P, P, i64, C.POINTER(KmeansCfg), i32, P, P, P, P]),
    "ecc_kmeans_assign_f32": (C.c_int, [P, P, i64, P, i32, C.c_float, P, P]),
    "ecc_kmeans_accumulate_xy16": (C.c_int, [P, P, i64, i64, P, P, i32, C.c_float, P, P, P]),
    "ecc_kmeans_update": (C.c_int, [P, P, P, i32, C.c_float, P, P]),
    "ecc_kmeans_labels_xy16": (C.c_int, [P, P, i64, i64, P, P, i32, C.c_float, P, P]),
    "ecc_kmeans_counts_xy16": (C.c_int, [P, P, i64, i64, P, i32, i32, P, P]),
    "ecc_kmeans_counts_status": (C.c_int, [P, P]),
    "ecc_kmeans_run_counts": (C.c_int, [P, P, i32, i32, C.POINTER(KmeansCfg), P, P, P]),
    "ecc_sae_max_combine": (C.c_int, [P, P, i32, i64, P, P]),
    "ecc_corner_cfg_default": (None, [C.POINTER(CornerCfg)]),
    "ecc_fast_detect": (C.c_int, [P, P, P, i64, C.POINTER(CornerCfg), P, P, P]),
    "ecc_fast_detect_nms": (C.c_int, [P, P, P, i64, C.POINTER(CornerCfg), P, P, i32, i32, P, P, P]),
    "ecc_fast_detect_prepare": (C.c_int, [P, P, P, i64, C.POINTER(CornerCfg), P, P]),
    "ecc_fast_detect_finish": (C.c_int, [P, P, P, i64, C.POINTER(CornerCfg), P, P, P]),
    "ecc_fast_detect_finish_nms": (C.c_int, [P, P, P, i64, C.POINTER(CornerCfg), P, P, i32, i32, P, P, P]),
    "ecc_fast_detect_status": (C.c_int, [P, P]),
    "ecc_fast_detect_stats": (C.c_int, [P, P, i32, P]),
    "ecc_sae_scatter": (C.c_int, [P, P, P, i64, i32, i32, P, P]),
    "ecc_corner_nms": (C.c_int, [P, P, P, i64, i32, i32, i32, i32, i32, P, P, P]),
    "ecc_corner_nms_status": (C.c_int, [P, P]),
    "ecc_corner_pack": (C.c_int, [P, P, P, i32, i32, P, P, P]),
    "ecc_tracker_update_lists": (C.c_int, [P, P, P, P, i32, P]),
    "ecc_tracker_cfg_default": (None, [C.POINTER(TrackerCfg)]),
    "ecc_tracker_create": (C.c_int, [P, C.POINTER(TrackerCfg), i32, i32, C.POINTER(P)]),
    "ecc_tracker_destroy": (C.c_int, [P]),
    "ecc_tracker_update": (C.c_int, [P, P, P, i32, i32, P]),
    "ecc_tracker_get_tracks": (C.c_int, [P, P, i32, C.POINTER(i32), P]),
    "ecc_tracker_get_groups": (C.c_int, [P, P, i32, C.POINTER(i32), P, i32, P]),
    "ecc_tracker_status": (C.c_int, [P, P]),
    "ecc_tracker_set_tracks": (C.c_int, [P, P, i32, i32, P]),
    "ecc_tracker_next_label": (C.c_int, [P, C.POINTER(i32), P]),
    "ecc_eps_counts": (C.c_int, [P, P, i64, i64, P, C.c_double, i32, P, P, P]),
    "ecc_eps_lists": (C.c_int, [P, P, i64, i64, P, C.c_double, P, P, P, i64, P]),
    "ecc_eps_total": (C.c_int, [P, P, i64, C.POINTER(i64), P]),
    "ecc_gen_cfg_default": (None, [C.POINTER(GenCfg)]),
    "ecc_gen_events": (C.c_int, [C.POINTER(GenCfg), i64, i64, P, P, P]),
    "ecc_fast_detect_status": (C.c_int, [P, P]),
    "ecc_read_csv": (i64, [C.c_char_p, P, P, P, i64]),
    "ecc_count_csv": (i64, [C.c_char_p]),
    "ecc_raw_probe": (C.c_int, [C.c_char_p, C.POINTER(RawInfo)]),
    "ecc_raw_read_words": (i64, [C.c_char_p, C.POINTER(RawInfo), i64, i64, P]),
    "ecc_evt_decode": (C.c_int, [P, i32, P, i64, P, P, P, i64, P, P, P]),
    "ecc_evt_status": (C.c_int, [P, P]),
    "ecc_evt_encode": (i64, [i32, P, P, P, i64, P, i64]),
    "ecc_radius_counts_f64": (C.c_int, [P, P, i64, i32, C.c_double, i32, P, P, P]),
    "ecc_radius_lists_f64": (C.c_int, [P, P, i64, i32, C.c_double, P, P, P, P, i64, P]),
    "ecc_radius_status": (C.c_int, [P, P]),
    "ecc_radius_counts_f32": (C.c_int, [P, P, i64, i32, C.c_double, i32, P, P, P]),
    "ecc_radius_lists_f32": (C.c_int, [P, P, i64, i32, C.c_double, P, P, P, P, i64, P]),
    "ecc_lists_sort_ascending": (C.c_int, [P, i64, P, i64, P, P, P]),
    "ecc_dbscan_cloud_f32": (C.c_int, [P, P, i64, i32, C.c_double, i32, i32, i32, P, P, P, i64, P, P]),
    "ecc_dbscan_cloud_f64": (C.c_int, [P, P, i64, i32, C.c_double, i32, i32, i32, P, P, P, i64, P, P]),
    "ecc_dbscan_cloud_status": (C.c_int, [P, P]),
    "ecc_optics_f64": (C.c_int, [P, P, i64, i32, i32, C.c_double, P, P, P]),
    "ecc_dbscan_extract": (C.c_int, [P, i64, i64, P, P, P, i64, i32, i32, i32, P, P, P, i64, P, P]),
    "ecc_dbscan_grid": (C.c_int, [P, P, i64, i64, P, C.c_double, i32, i32, i32, P, P, P, i64, P, P]),
    "ecc_dbscan_status": (C.c_int, [P, P]),
    "ecc_device_sync": (C.c_int, []),
    "ecc_reslice_n_us": (C.c_int, [P, P, i64, i64, P, i64, P, P]),
    "ecc_dist_available": (C.c_int, []),
    "ecc_dist_get_unique_id": (C.c_int, [P]),
    "ecc_dist_init": (C.c_int, [C.POINTER(P), P, P, i32, i32]),
    "ecc_dist_destroy": (C.c_int, [P]),
    "ecc_dist_rank": (C.c_int, [P, C.POINTER(i32), C.POINTER(i32)]),
    "ecc_dist_allreduce_counts": (C.c_int, [P, P, i64, P]),
    "ecc_dist_allreduce_f64_max": (C.c_int, [P, P, i64, P]),
    "ecc_dist_sae_handoff": (C.c_int, [P, P, i64, P, P, P]),
    "ecc_dist_gather_corners": (C.c_int, [P, P, P, i32, P, i64, P, P, i64, C.POINTER(i64), C.POINTER(i64), P]),
}
DIST_ID_BYTES = 128
for _name, (_res, _args) in _sigs.items():
    _f = getattr(lib, _name)  # every bound symbol must exist (fail loudly on a stale build)
    _f.restype = _res
    _f.argtypes = _args


def _ptr(a) -> int | None:
    if a is None:
        return None
    if isinstance(a, DeviceArray):
        return a.ptr
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a)


def device_count() -> int:
    n = C.c_int(0)
    lib.ecc_device_count(C.byref(n))
    return n.value


# ---------------------------------------------------------------- device memory
class DeviceArray:
    """A hipMalloc'd buffer with a numpy dtype/shape, freed on garbage collection."""

    def __init__(self, shape, dtype):
        self.shape = tuple(shape) if np.ndim(shape) else (int(shape),)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = P()
        check(lib.ecc_dev_alloc(C.byref(p), max(self.nbytes, 16)), "ecc_dev_alloc")
        self.ptr = p.value

    @classmethod
    def from_numpy(cls, a: np.ndarray, stream=None) -> "DeviceArray":
        a = np.ascontiguousarray(a)
        d = cls(a.shape, a.dtype)
        if a.nbytes:
            check(lib.ecc_memcpy_h2d(d.ptr, a.ctypes.data, a.nbytes, stream), "h2d")
            check(lib.ecc_stream_sync(stream))
        return d

    @classmethod
    def zeros(cls, shape, dtype, stream=None) -> "DeviceArray":
        d = cls(shape, dtype)
        check(lib.ecc_memset_async(d.ptr, 0, max(d.nbytes, 16), stream), "memset")
        check(lib.ecc_stream_sync(stream))
        return d

    def fill_bytes(self, value: int, stream=None):
        check(lib.ecc_memset_async(self.ptr, value, self.nbytes, stream), "memset")

    def numpy(self, stream=None) -> np.ndarray:
        """Copies to the host.  stream=None waits for ALL device work first (library streams are
        non-blocking, so the null stream alone does not order after them)."""
        out = np.empty(self.shape, self.dtype)
        if stream is None:
            check(lib.ecc_device_sync(), "ecc_device_sync")
        if self.nbytes:
            check(lib.ecc_memcpy_d2h(out.ctypes.data, self.ptr, self.nbytes, stream), "d2h")
        return out

    def copy_from(self, a: np.ndarray, stream=None):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        assert a.nbytes <= self.nbytes
        check(lib.ecc_memcpy_h2d(self.ptr, a.ctypes.data, a.nbytes, stream), "h2d")
        check(lib.ecc_stream_sync(stream))

    def __del__(self):
        if getattr(self, "ptr", None):
            lib.ecc_dev_free(self.ptr)
            self.ptr = None


class Context:
    """ecc_ctx + a private stream."""

    def __init__(self, device: int = 0, own_stream: bool = True, stream: int | None = None):
        check(lib.ecc_set_device(device), "ecc_set_device")
        p = P()
        check(lib.ecc_ctx_create(C.byref(p), device), "ecc_ctx_create")
        self.ctx = p.value
        self.device = device
        self.stream = None
        self._own_stream = False
        if stream is not None:  # an external hipStream_t (e.g. torch's current stream)
            self.stream = stream
        elif own_stream:
            s = P()
            check(lib.ecc_stream_create(C.byref(s)), "ecc_stream_create")
            self.stream = s.value
            self._own_stream = True

    def sync(self):
        check(lib.ecc_stream_sync(self.stream), "sync")

    # per-kernel timing (ecc_ctx_set_timing): HIP events around every launch of this context
    def set_timing(self, on: bool):
        check(lib.ecc_ctx_set_timing(self.ctx, 1 if on else 0), "ecc_ctx_set_timing")

    def timing_reset(self):
        check(lib.ecc_ctx_timing_reset(self.ctx), "ecc_ctx_timing_reset")

    def timing_report(self) -> dict:
        buf = C.create_string_buffer(1 << 16)
        check(lib.ecc_ctx_timing_report(self.ctx, buf, len(buf)), "ecc_ctx_timing_report")
        return json.loads(buf.value.decode())

    def last_error(self) -> str:
        return lib.ecc_ctx_last_error(self.ctx).decode()

    def close(self):
        if self.ctx:
            lib.ecc_ctx_destroy(self.ctx)
            self.ctx = None
        if self.stream and self._own_stream:
            lib.ecc_stream_destroy(self.stream)
        self.stream = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- 1. downsample
    def downsample_hash(self, xy: DeviceArray, n: int, cfg: HashCfg | None = None,
                        want_idx: bool = True):
        cfg = cfg or hash_cfg()
        nw = (n + cfg.window - 1) // cfg.window
        rep_xy = DeviceArray(max(nw * cfg.window, 1), np.uint32)
        rep_idx = DeviceArray(max(nw * cfg.window, 1), np.uint32) if want_idx else None
        uniq = DeviceArray(max(nw, 1), np.int32)
        rep = DeviceArray(max(nw, 1), np.int32)
        check(lib.ecc_downsample_hash(self.ctx, xy.ptr, n, C.byref(cfg), rep_xy.ptr,
                                      _ptr(rep_idx), uniq.ptr, rep.ptr, self.stream),
              "ecc_downsample_hash")
        return rep_xy, rep_idx, uniq, rep, nw

    def dedup_exact(self, xy: DeviceArray, n: int, window: int = 8192):
        """analyzeCoordinates per window: (uniq_idx, uniq_cnt, n_unique, n_windows)."""
        nw = (n + window - 1) // window
        idx = DeviceArray(max(nw * window, 1), np.uint32)
        cnt = DeviceArray(max(nw * window, 1), np.int32)
        u = DeviceArray(max(nw, 1), np.int32)
        check(lib.ecc_dedup_exact(self.ctx, xy.ptr, n, window, idx.ptr, cnt.ptr, u.ptr, self.stream),
              "ecc_dedup_exact")
        return idx, cnt, u, nw

    # ---- 2. k-means
    def kmeans_xy16(self, xy: DeviceArray, n_segs: int, stride: int, counts: DeviceArray | None,
                    centroids: DeviceArray, cfg: KmeansCfg, labels: DeviceArray | None = None,
                    iters: DeviceArray | None = None):
        check(lib.ecc_kmeans_run_xy16(self.ctx, xy.ptr, n_segs, stride, _ptr(counts),
                                      C.byref(cfg), centroids.ptr, _ptr(labels), _ptr(iters),
                                      self.stream), "ecc_kmeans_run_xy16")

    def kmeans_xy16_frame(self, xy: DeviceArray, n_segs: int, stride: int, counts: DeviceArray | None, w: int,
                          h: int, centroids: DeviceArray, cfg: KmeansCfg, labels: DeviceArray | None = None,
                          iters: DeviceArray | None = None):
        check(lib.ecc_kmeans_run_xy16_frame(self.ctx, xy.ptr, n_segs, stride, _ptr(counts), w, h, C.byref(cfg),
                                            centroids.ptr, _ptr(labels), _ptr(iters), self.stream),
              "ecc_kmeans_run_xy16_frame")

    def kmeans_f32(self, xy: DeviceArray, n: int, centroids: DeviceArray, cfg: KmeansCfg,
                   labels: DeviceArray | None = None, iters: DeviceArray | None = None):
        check(lib.ecc_kmeans_run_f32(self.ctx, xy.ptr, n, C.byref(cfg), centroids.ptr,
                                     _ptr(labels), _ptr(iters), self.stream), "ecc_kmeans_run_f32")

    def kmeans_f32_engine(self, xy: DeviceArray, n: int, centroids: DeviceArray, cfg: KmeansCfg, engine: int,
                          labels: DeviceArray | None = None, iters: DeviceArray | None = None):
        """engine: 0 default, 1 vector (SGPR centres), 2 matrix cores (4x4x1 MFMA distance + exact
        fallback), 3 matrix cores in the streaming 32x32x2 form (k <= 16, 16-B aligned points)."""
        check(lib.ecc_kmeans_run_f32_engine(self.ctx, xy.ptr, n, C.byref(cfg), engine, centroids.ptr,
                                            _ptr(labels), _ptr(iters), self.stream), "ecc_kmeans_run_f32_engine")

    def kmeans_assign_f32(self, xy: DeviceArray, n: int, centroids: DeviceArray, k: int,
                          thr: float, labels: DeviceArray):
        check(lib.ecc_kmeans_assign_f32(self.ctx, xy.ptr, n, centroids.ptr, k, thr, labels.ptr,
                                        self.stream), "ecc_kmeans_assign_f32")

    # ---- 3. SAE + arc corners
    def fast_detect(self, xy: DeviceArray, t: DeviceArray, n: int, cfg: CornerCfg,
                    sae: DeviceArray, flags: DeviceArray):
        check(lib.ecc_fast_detect(self.ctx, xy.ptr, t.ptr, n, C.byref(cfg), sae.ptr, flags.ptr,
                                  self.stream), "ecc_fast_detect")

    def fast_detect_nms(self, xy: DeviceArray, t: DeviceArray, n: int, cfg: CornerCfg, sae: DeviceArray,
                        flags: DeviceArray, box: int, cap: int, out: DeviceArray, counts: DeviceArray):
        """fast_detect then corner_nms over cfg's slices, with the flag pass writing the NMS
        candidate lists (FCT/…group_track.cpp:832-837: detect, then filterCorners per slice)."""
        check(lib.ecc_fast_detect_nms(self.ctx, xy.ptr, t.ptr, n, C.byref(cfg), sae.ptr, flags.ptr, box, cap,
                                      out.ptr, counts.ptr, self.stream), "ecc_fast_detect_nms")

    def fast_detect_status(self) -> int:
        return lib.ecc_fast_detect_status(self.ctx, self.stream)

    def fast_detect_stats(self) -> dict:
        out = np.zeros(4, np.int64)
        check(lib.ecc_fast_detect_stats(self.ctx, out.ctypes.data, 4, self.stream), "ecc_fast_detect_stats")
        return {"items": int(out[0]), "overflow_items": int(out[1]), "slices": int(out[2]), "groups": int(out[3])}

    def sae_scatter(self, xy: DeviceArray, t: DeviceArray, n: int, w: int, h: int,
                    sae: DeviceArray):
        check(lib.ecc_sae_scatter(self.ctx, xy.ptr, t.ptr, n, w, h, sae.ptr, self.stream),
              "ecc_sae_scatter")

    # ---- 4. NMS
    def corner_nms(self, xy: DeviceArray, flags: DeviceArray, n: int, slice_events: int, w: int,
                   h: int, box: int, cap: int, out: DeviceArray, counts: DeviceArray):
        check(lib.ecc_corner_nms(self.ctx, xy.ptr, flags.ptr, n, slice_events, w, h, box, cap,
                                 out.ptr, counts.ptr, self.stream), "ecc_corner_nms")

    def corner_pack(self, nms_out, counts, n_slices: int, cap: int, out, offsets):
        """Dense per-slice corner lists (DeviceArrays or raw device pointers)."""
        check(lib.ecc_corner_pack(self.ctx, _ptr(nms_out), _ptr(counts), n_slices, cap, _ptr(out), _ptr(offsets),
                                  self.stream), "ecc_corner_pack")

    def corner_nms_status(self) -> int:
        return lib.ecc_corner_nms_status(self.ctx, self.stream)

    # ---- 6. eps-neighbourhoods
    def eps_counts(self, xy: DeviceArray, n_segs: int, stride: int, counts_in, eps: float,
                   min_pts: int, counts: DeviceArray, core: DeviceArray | None):
        check(lib.ecc_eps_counts(self.ctx, xy.ptr, n_segs, stride, _ptr(counts_in), eps, min_pts,
                                 counts.ptr, _ptr(core), self.stream), "ecc_eps_counts")

    def eps_lists(self, xy: DeviceArray, n_segs: int, stride: int, counts_in, eps: float,
                  counts: DeviceArray, offsets: DeviceArray, nbr: DeviceArray, nbr_cap: int):
        check(lib.ecc_eps_lists(self.ctx, xy.ptr, n_segs, stride, _ptr(counts_in), eps,
                                counts.ptr, offsets.ptr, nbr.ptr, nbr_cap, self.stream),
              "ecc_eps_lists")


    def dbscan_extract(self, n_segs: int, stride: int, counts_in, offsets: DeviceArray, nbr: DeviceArray,
                       min_pts: int, min_size: int, max_size: int, labels: DeviceArray, n_clusters: DeviceArray,
                       dups: DeviceArray | None, dup_cap: int, n_dups: DeviceArray):
        check(lib.ecc_dbscan_extract(self.ctx, n_segs, stride, _ptr(counts_in), offsets.ptr, nbr.ptr,
                                     nbr.nbytes // 4, min_pts,
                                     min_size, max_size, labels.ptr, n_clusters.ptr, _ptr(dups), dup_cap,
                                     n_dups.ptr, self.stream), "ecc_dbscan_extract")

    def dbscan_grid(self, xy: DeviceArray, n_segs: int, stride: int, counts_in, eps: float, min_pts: int,
                    min_size: int, max_size: int, labels: DeviceArray, n_clusters: DeviceArray,
                    dups: DeviceArray | None, dup_cap: int, n_dups: DeviceArray):
        check(lib.ecc_dbscan_grid(self.ctx, xy.ptr, n_segs, stride, _ptr(counts_in), eps, min_pts, min_size,
                                  max_size, labels.ptr, n_clusters.ptr, _ptr(dups), dup_cap, n_dups.ptr,
                                  self.stream), "ecc_dbscan_grid")

    def radius_counts_f64(self, pts: DeviceArray, n: int, dim: int, eps: float, min_pts: int,
                          counts: DeviceArray, core: DeviceArray | None = None):
        check(lib.ecc_radius_counts_f64(self.ctx, pts.ptr, n, dim, eps, min_pts, counts.ptr, _ptr(core),
                                        self.stream), "ecc_radius_counts_f64")

    def radius_lists_f64(self, pts: DeviceArray, n: int, dim: int, eps: float, counts: DeviceArray,
                         offsets: DeviceArray, nbr: DeviceArray | None, nbr_cap: int,
                         nbr_dist: DeviceArray | None = None):
        check(lib.ecc_radius_lists_f64(self.ctx, pts.ptr, n, dim, eps, counts.ptr, offsets.ptr, _ptr(nbr),
                                       _ptr(nbr_dist), nbr_cap, self.stream), "ecc_radius_lists_f64")

    def radius_status(self) -> int:
        return lib.ecc_radius_status(self.ctx, self.stream)

    def radius_counts_f32(self, pts: DeviceArray, n: int, dim: int, eps: float, min_pts: int,
                          counts: DeviceArray, core: DeviceArray | None = None):
        check(lib.ecc_radius_counts_f32(self.ctx, pts.ptr, n, dim, eps, min_pts, counts.ptr, _ptr(core),
                                        self.stream), "ecc_radius_counts_f32")

    def radius_lists_f32(self, pts: DeviceArray, n: int, dim: int, eps: float, counts: DeviceArray,
                         offsets: DeviceArray, nbr: DeviceArray | None, nbr_cap: int,
                         nbr_dist: DeviceArray | None = None):
        check(lib.ecc_radius_lists_f32(self.ctx, pts.ptr, n, dim, eps, counts.ptr, offsets.ptr, _ptr(nbr),
                                       _ptr(nbr_dist), nbr_cap, self.stream), "ecc_radius_lists_f32")

    def lists_sort_ascending(self, n: int, offsets: DeviceArray, total: int, nbr: DeviceArray,
                             nbr_dist: DeviceArray | None = None):
        check(lib.ecc_lists_sort_ascending(self.ctx, n, offsets.ptr, total, nbr.ptr, _ptr(nbr_dist), self.stream),
              "ecc_lists_sort_ascending")

    def dbscan_cloud(self, pts: DeviceArray, n: int, dim: int, eps: float, min_pts: int, min_size: int,
                     max_size: int, labels: DeviceArray, n_clusters: DeviceArray, dups: DeviceArray | None,
                     dup_cap: int, n_dups: DeviceArray):
        """DBSCAN of one cloud (device float32 or float64 [n*dim], picked by pts.dtype)."""
        fn = lib.ecc_dbscan_cloud_f32 if pts.dtype == np.float32 else lib.ecc_dbscan_cloud_f64
        check(fn(self.ctx, pts.ptr, n, dim, eps, min_pts, min_size, max_size, labels.ptr, n_clusters.ptr,
                 _ptr(dups), dup_cap, n_dups.ptr, self.stream), "ecc_dbscan_cloud")

    def dbscan_cloud_status(self) -> int:
        return lib.ecc_dbscan_cloud_status(self.ctx, self.stream)

    def optics_f64(self, pts_host, min_pts: int, eps: float = -1.0):
        """OPTICS ordering of host points (n x dim, dim 1-3): (order int64[n], reach double[n])."""
        pts = np.ascontiguousarray(pts_host, np.float64)
        n, dim = pts.shape
        order = np.zeros(n, np.int64)
        reach = np.zeros(n, np.float64)
        check(lib.ecc_optics_f64(self.ctx, pts.ctypes.data, n, dim, min_pts, eps, order.ctypes.data,
                                 reach.ctypes.data, self.stream), "ecc_optics_f64")
        return order, reach

    def dbscan_status(self) -> int:
        return lib.ecc_dbscan_status(self.ctx, self.stream)

    # ---- 8. RAW ingest
    def evt_decode(self, fmt: int, words: DeviceArray, n_words: int, xy: DeviceArray | None,
                   t: DeviceArray | None, p: DeviceArray | None, cap: int, n_out: DeviceArray,
                   state: DeviceArray | None = None):
        check(lib.ecc_evt_decode(self.ctx, fmt, words.ptr, n_words, _ptr(xy), _ptr(t), _ptr(p), cap,
                                 n_out.ptr, _ptr(state), self.stream), "ecc_evt_decode")

    def evt_status(self) -> int:
        return lib.ecc_evt_status(self.ctx, self.stream)

    def reslice_n_us(self, t: DeviceArray, n: int, period_us: int, bounds: DeviceArray,
                     max_slices: int, n_slices: DeviceArray):
        check(lib.ecc_reslice_n_us(self.ctx, t.ptr, n, period_us, bounds.ptr, max_slices,
                                   n_slices.ptr, self.stream), "ecc_reslice_n_us")


class Tracker:
    """Device-resident CornerTracker (FCT/…group_track.cpp:201-537)."""

    def __init__(self, ctx: Context, cfg: TrackerCfg | None = None, max_tracks: int = 4096,
                 max_detections: int = 4096):
        self.ctx = ctx
        self.cfg = cfg or tracker_cfg()
        p = P()
        check(lib.ecc_tracker_create(ctx.ctx, C.byref(self.cfg), max_tracks, max_detections,
                                     C.byref(p)), "ecc_tracker_create")
        self.tr = p.value
        self.max_tracks = max_tracks

    def update(self, corners: DeviceArray, counts: DeviceArray, n_slices: int, cap: int):
        check(lib.ecc_tracker_update(self.tr, corners.ptr, counts.ptr, n_slices, cap,
                                     self.ctx.stream), "ecc_tracker_update")

    def update_lists(self, corners, starts, counts, n_slices: int):
        """Slice s = corners[starts[s] .. starts[s] + counts[s]) (device pointers or DeviceArrays)."""
        check(lib.ecc_tracker_update_lists(self.tr, _ptr(corners), _ptr(starts), _ptr(counts), n_slices,
                                           self.ctx.stream), "ecc_tracker_update_lists")

    def status(self) -> int:
        return lib.ecc_tracker_status(self.tr, self.ctx.stream)

    def tracks(self):
        buf = (Track * self.max_tracks)()
        n = i32(0)
        rc = lib.ecc_tracker_get_tracks(self.tr, buf, self.max_tracks, C.byref(n), self.ctx.stream)
        if rc not in (OK, ERR_CAPACITY):
            check(rc, "ecc_tracker_get_tracks")
        return [buf[i] for i in range(min(n.value, self.max_tracks))]

    def groups(self):
        cap = self.max_tracks
        buf = (Group * cap)()
        labels = np.zeros(cap, np.int32)
        n = i32(0)
        rc = lib.ecc_tracker_get_groups(self.tr, buf, cap, C.byref(n), labels.ctypes.data, cap,
                                        self.ctx.stream)
        if rc not in (OK, ERR_CAPACITY):
            check(rc, "ecc_tracker_get_groups")
        return [buf[i] for i in range(min(n.value, cap))], labels

    def next_label(self) -> int:
        v = i32(0)
        check(lib.ecc_tracker_next_label(self.tr, C.byref(v), self.ctx.stream), "ecc_tracker_next_label")
        return v.value

    def set_tracks(self, tracks, next_label: int):
        """Replace the state by a track list (e.g. another tracker's tracks()) and next label."""
        arr = (Track * max(len(tracks), 1))(*tracks)
        check(lib.ecc_tracker_set_tracks(self.tr, arr, len(tracks), next_label, self.ctx.stream),
              "ecc_tracker_set_tracks")

    def close(self):
        if self.tr:
            lib.ecc_tracker_destroy(self.tr)
            self.tr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Timer:
    """HIP-event timer on a given stream (measures exactly the work queued on that stream)."""

    def __init__(self, stream=None):
        self.stream = stream
        a, b = P(), P()
        check(lib.ecc_event_create(C.byref(a)))
        check(lib.ecc_event_create(C.byref(b)))
        self.a, self.b = a.value, b.value

    def start(self):
        check(lib.ecc_event_record(self.a, self.stream))

    def stop(self) -> float:
        check(lib.ecc_event_record(self.b, self.stream))
        ms = C.c_float(0)
        check(lib.ecc_event_elapsed_ms(C.byref(ms), self.a, self.b))
        return ms.value

    def __del__(self):
        try:
            lib.ecc_event_destroy(self.a)
            lib.ecc_event_destroy(self.b)
        except Exception:
            pass


# ---------------------------------------------------------------- config helpers
def hash_cfg(**kw) -> HashCfg:
    c = HashCfg()
    lib.ecc_hash_cfg_default(C.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def kmeans_cfg(**kw) -> KmeansCfg:
    c = KmeansCfg()
    lib.ecc_kmeans_cfg_default(C.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def corner_cfg(**kw) -> CornerCfg:
    c = CornerCfg()
    lib.ecc_corner_cfg_default(C.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def tracker_cfg(**kw) -> TrackerCfg:
    c = TrackerCfg()
    lib.ecc_tracker_cfg_default(C.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def gen_cfg(**kw) -> GenCfg:
    c = GenCfg()
    lib.ecc_gen_cfg_default(C.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def gen_events(n: int, first: int = 0, **kw):
    """Synthetic event stream (host numpy arrays xy:u32, t:i64, p:u8)."""
    cfg = gen_cfg(**kw)
    xy = np.empty(n, np.uint32)
    t = np.empty(n, np.int64)
    p = np.empty(n, np.uint8)
    check(lib.ecc_gen_events(C.byref(cfg), first, n, xy.ctypes.data, t.ctypes.data,
                             p.ctypes.data), "ecc_gen_events")
    return xy, t, p


def read_csv(path: str):
    n = lib.ecc_count_csv(str(path).encode())
    if n < 0:
        raise EccError(int(n), f"read_csv({path})")
    xy = np.empty(n, np.uint32)
    t = np.empty(n, np.int64)
    p = np.empty(n, np.uint8)
    got = lib.ecc_read_csv(str(path).encode(), xy.ctypes.data, t.ctypes.data, p.ctypes.data, n)
    return xy[:got], t[:got], p[:got]


EVT2, EVT3 = 2, 3
EVT_STATE_BYTES = 64


def raw_probe(path) -> RawInfo:
    info = RawInfo()
    check(lib.ecc_raw_probe(str(path).encode(), C.byref(info)), f"raw_probe({path})")
    return info


def raw_read_words(path, info: RawInfo, first: int = 0, n: int | None = None) -> np.ndarray:
    n = info.n_words - first if n is None else n
    out = np.empty(max(n, 0), np.uint32 if info.format == EVT2 else np.uint16)
    got = lib.ecc_raw_read_words(str(path).encode(), C.byref(info), first, n, out.ctypes.data)
    if got < 0:
        raise EccError(int(got), f"raw_read_words({path})")
    return out[:got]


def evt_encode(fmt: int, xy, t, p) -> np.ndarray:
    """RAW writer (ecc_evt_encode): events -> EVT 2.0 (u32) / EVT 3.0 (u16) words."""
    xy = np.ascontiguousarray(xy, np.uint32)
    t = np.ascontiguousarray(t, np.int64)
    p = np.ascontiguousarray(p, np.uint8)
    n = len(xy)
    cap = 2 * n + 1 if fmt == EVT2 else 4 * n + 4 + (2 * int(t[-1] >> 24) if n else 0)
    out = np.empty(max(cap, 1), np.uint32 if fmt == EVT2 else np.uint16)
    k = lib.ecc_evt_encode(fmt, xy.ctypes.data, t.ctypes.data, p.ctypes.data, n, out.ctypes.data, cap)
    if k < 0:
        raise EccError(int(k), "evt_encode")
    return out[:k].copy()


def pack_xy(x, y) -> np.ndarray:
    return (np.asarray(x, np.uint32) & 0xFFFF) | ((np.asarray(y, np.uint32) & 0xFFFF) << 16)


def unpack_xy(xy):
    xy = np.asarray(xy, np.uint32)
    return (xy & 0xFFFF).astype(np.int32), (xy >> 16).astype(np.int32)


class Dist:
    """Native RCCL communicator of one rank (ecc_dist_*: librccl opened by libecc, collectives on
    the caller's stream).  `uid` is the 128-byte id rank 0 made with unique_id(), shipped to the
    other ranks over any channel."""

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * DIST_ID_BYTES)()
        check(lib.ecc_dist_get_unique_id(buf), "ecc_dist_get_unique_id")
        return bytes(buf)

    def __init__(self, ctx: "Context", uid: bytes, n_ranks: int, rank: int):
        self.ctx = ctx
        self.d = P()
        buf = (C.c_uint8 * DIST_ID_BYTES).from_buffer_copy(uid)
        rc = lib.ecc_dist_init(C.byref(self.d), ctx.ctx, buf, n_ranks, rank)
        if rc != OK:
            raise EccError(rc, f"ecc_dist_init: {lib.ecc_ctx_last_error(ctx.ctx).decode()}")

    def allreduce_counts(self, ptr: int, n: int, stream=None):
        check(lib.ecc_dist_allreduce_counts(self.d, ptr, n, stream if stream is not None else self.ctx.stream),
              "ecc_dist_allreduce_counts")

    def allreduce_f64_max(self, ptr: int, n: int, stream=None):
        check(lib.ecc_dist_allreduce_f64_max(self.d, ptr, n, stream if stream is not None else self.ctx.stream),
              "ecc_dist_allreduce_f64_max")

    def sae_handoff(self, local_ptr: int, hw: int, all_ptr: int, sae_ptr: int, stream=None):
        check(lib.ecc_dist_sae_handoff(self.d, local_ptr, hw, all_ptr, sae_ptr,
                                       stream if stream is not None else self.ctx.stream), "ecc_dist_sae_handoff")

    def gather_corners(self, packed_ptr: int, offsets_ptr: int, n_slices: int, stream=None):
        """-> (all DeviceArray[CORNER_DTYPE], starts DeviceArray[int64], counts DeviceArray[int32],
        n_slices_total): the arguments of ecc_tracker_update_lists over every rank's lists."""
        st = stream if stream is not None else self.ctx.stream
        ns_tot, stride = i64(0), i64(0)
        check(lib.ecc_dist_gather_corners(self.d, packed_ptr, offsets_ptr, n_slices, None, 0, None, None, 0,
                                          C.byref(ns_tot), C.byref(stride), st), "ecc_dist_gather_corners(sizes)")
        nr = i32(0)
        check(lib.ecc_dist_rank(self.d, None, C.byref(nr)))
        cap = nr.value * stride.value
        all_ = DeviceArray(max(cap, 1), CORNER_DTYPE)
        starts = DeviceArray(max(ns_tot.value, 1), np.int64)
        counts = DeviceArray(max(ns_tot.value, 1), np.int32)
        check(lib.ecc_dist_gather_corners(self.d, packed_ptr, offsets_ptr, n_slices, all_.ptr, cap, starts.ptr,
                                          counts.ptr, ns_tot.value, C.byref(ns_tot), C.byref(stride), st),
              "ecc_dist_gather_corners")
        return all_, starts, counts, ns_tot.value

    def close(self):
        if self.d:
            lib.ecc_dist_destroy(self.d)
            self.d = P()
