"""Tracker state export / import (ecc_tracker_next_label + ecc_tracker_set_tracks): the
reference's CornerTracker is a copyable value (FCT/metavision_time_surface_periodic_group_track.cpp
:163-199), which SURVEY §5 (checkpoint / resume) and §8e (track state handed rank -> rank) need.
A tracker restored from another's state continues exactly like the uninterrupted one."""
import numpy as np
import pytest

from parity import group_key, track_key

pytestmark = pytest.mark.gpu


def dev(ecc, a):
    return ecc.DeviceArray.from_numpy(np.ascontiguousarray(a))


def _update(ecc, gpu, tr, d_out, d_cnt, s0, s1, cap):
    ecc.check(ecc.lib.ecc_tracker_update(tr.tr, d_out.ptr + s0 * cap * 12, d_cnt.ptr + s0 * 4, s1 - s0, cap,
                                         gpu.stream), "ecc_tracker_update")


@pytest.mark.parametrize("cut", [3, 17, 35])
def test_tracker_checkpoint_round_trip_continues_identically(ecc, orc, gpu, cut):
    W, H, ns, cap = 346, 260, 36, 4096
    n = 16384 * ns
    xy, t, _ = ecc.gen_events(n, seed=23, width=W, height=H)
    o_flags, _ = orc.fast_detect(xy, t, W, H)
    o_out, o_cnt, _ = orc.corner_nms(xy, o_flags, W, H, cap=cap)
    d_out, d_cnt = dev(ecc, o_out), dev(ecc, o_cnt)
    full = ecc.Tracker(gpu)
    _update(ecc, gpu, full, d_out, d_cnt, 0, ns, cap)
    a = ecc.Tracker(gpu)
    _update(ecc, gpu, a, d_out, d_cnt, 0, cut, cap)
    state, nl = a.tracks(), a.next_label()
    assert nl >= len(state) > 0
    b = ecc.Tracker(gpu)
    b.set_tracks(state, nl)
    assert [track_key(x) for x in b.tracks()] == [track_key(x) for x in state]
    assert b.next_label() == nl and b.groups()[0] == []
    _update(ecc, gpu, b, d_out, d_cnt, cut, ns, cap)
    assert b.status() == 0 and full.status() == 0
    assert [track_key(x) for x in b.tracks()] == [track_key(x) for x in full.tracks()]
    (gb, lb), (gf, lf) = b.groups(), full.groups()
    assert [group_key(g) for g in gb] == [group_key(g) for g in gf] and len(gf) > 0
    assert np.array_equal(lb, lf)
    assert b.next_label() == full.next_label()
    # and the oracle over the whole stream
    otr = orc.OracleTracker(ecc.tracker_cfg())
    for s in range(ns):
        otr.update(o_out[s * cap: s * cap + o_cnt[s]])
    assert [track_key(x) for x in b.tracks()] == [track_key(x) for x in otr.tracks(ecc.Track)]


def test_tracker_set_tracks_rejects_bad_state(ecc, gpu):
    tr = ecc.Tracker(gpu, max_tracks=4)
    t = ecc.Track()
    t.hist_len = 17  # > ECC_TRACK_HIST_MAX
    assert ecc.lib.ecc_tracker_set_tracks(tr.tr, (ecc.Track * 1)(t), 1, 0, gpu.stream) == ecc.ERR_INVALID
    five = (ecc.Track * 5)()
    assert ecc.lib.ecc_tracker_set_tracks(tr.tr, five, 5, 0, gpu.stream) == ecc.ERR_CAPACITY
    tr.set_tracks([], 42)
    assert tr.tracks() == [] and tr.next_label() == 42
