"""Output comparison helpers — TEST INFRASTRUCTURE ONLY (tests/, bench.py's cpu_baseline/parity leg).

Every comparison is exact: integer outputs element for element, fp32 outputs by bit pattern
(the device arithmetic follows the oracle's operation order)."""
from __future__ import annotations

import numpy as np


def f32_bits(v) -> int:
    return int(np.float32(v).view(np.uint32))


def track_key(tr):
    """All state of a TrackedCorner (ecc_track / oracle track), fp32 fields as bit patterns."""
    return (tr.x, tr.y, tr.label, tr.frame_count, tr.is_matched, tr.frames_since_last_detection,
            tr.hist_len, tuple(tr.hist_x[:tr.hist_len]), tuple(tr.hist_y[:tr.hist_len]),
            f32_bits(tr.vx), f32_bits(tr.vy), f32_bits(tr.dir_cur_x), f32_bits(tr.dir_cur_y),
            f32_bits(tr.dir_tgt_x), f32_bits(tr.dir_tgt_y), tr.group_id)


def group_key(g):
    return (g.id, g.n_labels, g.first_label_offset, f32_bits(g.avg_vx), f32_bits(g.avg_vy),
            f32_bits(g.cx), f32_bits(g.cy), f32_bits(g.radius))


def tracker_mismatches(g_tracks, o_tracks, g_groups=None, o_groups=None) -> int:
    """Number of differing tracks (+ groups, + 1 per list-length difference)."""
    bad = abs(len(g_tracks) - len(o_tracks))
    bad += sum(track_key(a) != track_key(b) for a, b in zip(g_tracks, o_tracks))
    if g_groups is not None:
        bad += abs(len(g_groups) - len(o_groups))
        bad += sum(group_key(a) != group_key(b) for a, b in zip(g_groups, o_groups))
    return int(bad)


def windowed_mismatches(g, o, counts, stride) -> int:
    """Differing valid slots of a windowed (segmented) output: slot w*stride + k, k < counts[w]."""
    valid = (np.arange(stride)[None, :] < np.asarray(counts)[:, None]).ravel()
    n = len(valid)
    return int(np.count_nonzero(np.asarray(g)[:n][valid] != np.asarray(o)[:n][valid]))


def nms_mismatches(g_out, g_cnt, o_out, o_cnt, cap) -> tuple[int, int]:
    """(slices whose kept-corner lists differ, corners compared)."""
    g_out = np.asarray(g_out).view(np.int32).reshape(-1, cap, 3)
    o_out = np.asarray(o_out).view(np.int32).reshape(-1, cap, 3)
    bad = 0
    for s in range(len(o_cnt)):
        c = int(o_cnt[s])
        if int(g_cnt[s]) != c or not np.array_equal(g_out[s, :c], o_out[s, :c]):
            bad += 1
    return bad, int(np.sum(o_cnt))
