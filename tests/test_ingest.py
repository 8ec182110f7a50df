"""RAW event ingest: EVT 2.0 / EVT 3.0 decoding and the n-µs reslicer.

The reference opens every recording with Metavision::Camera::from_file(argv[1])
(FCT/…group_track.cpp:756-760) and slices with EventBufferReslicerAlgorithm (:772-774,
DSA/…opencl_store.cpp:351).  OpenEB is not vendored and ships no fixtures, so parity is
"unpinned" against it: the oracle restates the published word formats, its encoder and
decoder must round-trip exactly (CPU tests), and the HIP decoders must match the oracle
decoder bit for bit on the same words (GPU tests)."""
import numpy as np
import pytest

SENSOR = (1280, 720)


def events_random(n, seed, t_span=1 << 22, wh=SENSOR):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, wh[0], n)
    y = rng.integers(0, wh[1], n)
    t = np.sort(rng.integers(0, t_span, n)).astype(np.int64)
    p = rng.integers(0, 2, n).astype(np.uint8)
    return (x | (y << 16)).astype(np.uint32), t, p


def events_rows(n_runs, seed, wh=SENSOR):
    """Row bursts: runs of equal (t, y, p) with strictly increasing x (vector words)."""
    rng = np.random.default_rng(seed)
    xs, ys, ts, ps = [], [], [], []
    t = int(rng.integers(0, 1000))
    for _ in range(n_runs):
        t += int(rng.integers(0, 40))
        y, p = int(rng.integers(0, wh[1])), int(rng.integers(0, 2))
        x0 = int(rng.integers(0, wh[0] - 64))
        m = int(rng.integers(1, 30))
        x = np.unique(x0 + rng.integers(0, 60, m))
        xs.append(x); ys.append(np.full(len(x), y)); ts.append(np.full(len(x), t)); ps.append(np.full(len(x), p))
    x, y = np.concatenate(xs), np.concatenate(ys)
    return ((x | (y << 16)).astype(np.uint32), np.concatenate(ts).astype(np.int64),
            np.concatenate(ps).astype(np.uint8))


def concat(*evs):
    xy = np.concatenate([e[0] for e in evs])
    t = np.concatenate([e[1] for e in evs])
    p = np.concatenate([e[2] for e in evs])
    o = np.argsort(t, kind="stable")
    return xy[o], t[o], p[o]


# ------------------------------------------------------------------------------ CPU: oracle
@pytest.mark.parametrize("fmt", [2, 3])
@pytest.mark.parametrize("case", ["random", "rows", "loops", "noise"])
def test_oracle_evt_roundtrip(orc, fmt, case):
    if case == "random":
        ev = events_random(20000, 1)
    elif case == "rows":
        ev = events_rows(2000, 2)
    elif case == "loops":  # EVT 3.0 24-bit time loops (t up to 2^27)
        ev = concat(events_random(5000, 3, t_span=1 << 27), events_rows(500, 4))
    else:
        ev = concat(events_random(5000, 5), events_rows(500, 6))
    words = orc.evt_encode(fmt, *ev, seed=7, noise_pct=30 if case == "noise" else 5)
    xy, t, p = orc.evt_decode(fmt, words)
    assert len(xy) == len(ev[0])
    assert (xy == ev[0]).all() and (t == ev[1]).all() and (p == ev[2]).all()
    if fmt == 3 and case == "rows":  # the stream really uses vector words
        ty = words >> 12
        assert (ty == 4).sum() > 100 and (ty == 5).sum() > 100 and (ty == 3).sum() > 100


def test_oracle_evt3_known_words(orc):
    """Hand-assembled EVT 3.0 words (format table in include/ecc.h §8)."""
    w = np.array([
        0x8000 | 0x001,          # TIME_HIGH 1
        0x6000 | 0x023,          # TIME_LOW 0x23   -> t = 1<<12 | 0x23 = 4131
        0x0000 | 17,             # ADDR_Y 17
        0x2000 | (1 << 11) | 5,  # ADDR_X x=5 p=1
        0xA000 | 0x0FF,          # EXT_TRIGGER: no CD event
        0x3000 | 100,            # VECT_BASE_X 100 p=0
        0x4000 | 0b100000000101, # VECT_12: x 100, 102, 111
        0x5000 | 0b10000001,     # VECT_8 (base 112): x 112, 119
        0x2000 | 7,              # ADDR_X x=7 p=0
        0x8000 | 0x000,          # TIME_HIGH 0 < 1: one loop
        0x2000 | 9,              # t = 1<<24 | 0<<12 | 0x23
    ], np.uint16)
    xy, t, p = orc.evt_decode(3, w)
    x, y = xy & 0xFFFF, xy >> 16
    assert list(x) == [5, 100, 102, 111, 112, 119, 7, 9]
    assert (y == 17).all()
    assert list(p) == [1, 0, 0, 0, 0, 0, 0, 0]
    assert list(t) == [4131] * 7 + [(1 << 24) | 0x23]


def test_oracle_evt2_known_words(orc):
    w = np.array([
        0x1 << 28 | 5 << 22 | 3 << 11 | 4,  # CD_ON before any TIME_HIGH: t = 5
        0x8 << 28 | 10,                     # TIME_HIGH 10
        0x0 << 28 | 63 << 22 | 2047 << 11 | 2047,  # CD_OFF x=y=2047, t = 10<<6 | 63
        0xE << 28 | 12345,                  # OTHERS
    ], np.uint32)
    xy, t, p = orc.evt_decode(2, w)
    assert list(xy & 0xFFFF) == [3, 2047] and list(xy >> 16) == [4, 2047]
    assert list(t) == [5, (10 << 6) | 63] and list(p) == [1, 0]


def test_oracle_reslice(orc):
    rng = np.random.default_rng(3)
    t = np.sort(rng.integers(10_000, 400_000, 5000)).astype(np.int64)
    t[100:200] = t[100]                              # equal timestamps
    t = np.sort(np.concatenate([t, [1_000_000]]))    # a long gap -> empty slices
    for period in (1, 777, 50_000):
        bounds, ns = orc.reslice_n_us(t, period)
        base = (t[0] // period) * period
        edges = base + period * np.arange(ns)
        assert ns == (t[-1] - base) // period + 1
        assert (bounds[:ns] == np.searchsorted(t, edges, side="left")).all() and bounds[ns] == len(t)


def test_raw_probe_and_read(ecc, orc, tmp_path):
    """Host RAW reader (libecc, no GPU needed): header keys, payload offset, word reads."""
    ev = events_random(3000, 9)
    for fmt, hdr in [(3, "% date 2024-01-01\n% evt 3.0\n% format EVT3;height=720;width=1280\n% end\n"),
                     (2, "% geometry 640x480\n% evt 2.0\n% serial_number 00ca\n")]:
        words = orc.evt_encode(fmt, *ev, seed=1)
        path = tmp_path / f"rec{fmt}.raw"
        path.write_bytes(hdr.encode() + words.tobytes())
        info = ecc.raw_probe(path)
        assert info.format == fmt and info.word_bytes == (4 if fmt == 2 else 2)
        assert info.header_bytes == len(hdr) and info.n_words == len(words)
        assert (info.width, info.height) == ((1280, 720) if fmt == 3 else (640, 480))
        assert (ecc.raw_read_words(path, info) == words).all()
        assert (ecc.raw_read_words(path, info, 100, 50) == words[100:150]).all()
    bad = tmp_path / "bad.raw"
    bad.write_bytes(b"% evt 4.0\n% end\n\x00\x00")
    with pytest.raises(ecc.EccError):
        ecc.raw_probe(bad)


# ------------------------------------------------------------------------------ GPU parity
def _gpu_decode(ecc, gpu, fmt, words, cap=None, pieces=None, offset=0):
    """Decodes `words` on the GPU (optionally in pieces with a carry state, or from a
    misaligned start `offset` words into the buffer)."""
    n = len(words)
    cap = n * (1 if fmt == 2 else 12) if cap is None else cap
    buf = np.concatenate([np.zeros(offset, words.dtype), words]) if offset else words
    d_words = ecc.DeviceArray.from_numpy(buf if len(buf) else np.zeros(1, words.dtype))
    d_xy = ecc.DeviceArray(max(cap, 1), np.uint32)
    d_t = ecc.DeviceArray(max(cap, 1), np.int64)
    d_p = ecc.DeviceArray(max(cap, 1), np.uint8)
    d_n = ecc.DeviceArray(1, np.int64)
    wsz = words.dtype.itemsize
    if pieces is None:
        ptr = d_words.ptr + offset * wsz
        ecc.check(ecc.lib.ecc_evt_decode(gpu.ctx, fmt, ptr, n, d_xy.ptr, d_t.ptr, d_p.ptr, cap, d_n.ptr,
                                         None, gpu.stream))
        st = gpu.evt_status()
        gpu.sync()
        k = int(d_n.numpy()[0])
        m = min(k, cap)
        return d_xy.numpy()[:m], d_t.numpy()[:m], d_p.numpy()[:m], k, st
    state = ecc.DeviceArray.from_numpy(np.zeros(ecc.EVT_STATE_BYTES, np.uint8))
    outs, lo = [], 0
    for hi in [int(c) for c in pieces] + [n]:
        m = hi - lo
        ecc.check(ecc.lib.ecc_evt_decode(gpu.ctx, fmt, d_words.ptr + lo * wsz, m, d_xy.ptr, d_t.ptr, d_p.ptr,
                                         cap, d_n.ptr, state.ptr, gpu.stream))
        gpu.sync()
        k = int(d_n.numpy()[0])
        outs.append((d_xy.numpy()[:k], d_t.numpy()[:k], d_p.numpy()[:k]))
        lo = hi
    return (np.concatenate([o[0] for o in outs]), np.concatenate([o[1] for o in outs]),
            np.concatenate([o[2] for o in outs]), None, 0)


def _check_same(got, ref):
    assert len(got[0]) == len(ref[0])
    assert (got[0] == ref[0]).all() and (got[1] == ref[1]).all() and (got[2] == ref[2]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [2, 3])
@pytest.mark.parametrize("case", ["random", "rows", "loops", "noise"])
def test_gpu_evt_decode_matches_oracle(ecc, orc, gpu, fmt, case):
    if case == "random":
        ev = events_random(300_000, 11)
    elif case == "rows":
        ev = events_rows(20_000, 12)
    elif case == "loops":
        ev = concat(events_random(100_000, 13, t_span=1 << 28), events_rows(5000, 14))
    else:
        ev = concat(events_random(50_000, 15), events_rows(5000, 16))
    words = orc.evt_encode(fmt, *ev, seed=3, noise_pct=40 if case == "noise" else 5)
    ref = orc.evt_decode(fmt, words)
    _check_same(ref, ev)
    got = _gpu_decode(ecc, gpu, fmt, words)
    assert got[3] == len(ref[0]) and got[4] == 0
    _check_same(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [2, 3])
def test_gpu_evt_edges(ecc, orc, gpu, fmt):
    """Tiny and ragged buffers, chunk-boundary sizes, misaligned starts, arbitrary words."""
    ev = concat(events_random(30_000, 21), events_rows(3000, 22))
    words = orc.evt_encode(fmt, *ev, seed=5)
    for n in (0, 1, 2, 15, 16, 17, 31, 32, 33, 4095, 4096, 4097, 8191, 8192, 8193, 3 * 8192 + 5):
        w = words[:n]
        got = _gpu_decode(ecc, gpu, fmt, w)
        _check_same(got, orc.evt_decode(fmt, w))
    for off in (1, 3, 5):
        got = _gpu_decode(ecc, gpu, fmt, words, offset=off)
        _check_same(got, orc.evt_decode(fmt, words))
    # arbitrary (invalid-looking) words decode exactly as the sequential state machine
    rng = np.random.default_rng(fmt)
    junk = rng.integers(0, 1 << (32 if fmt == 2 else 16), 100_003, dtype=np.uint64).astype(
        np.uint32 if fmt == 2 else np.uint16)
    _check_same(_gpu_decode(ecc, gpu, fmt, junk), orc.evt_decode(fmt, junk))


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [2, 3])
def test_gpu_evt_streaming_state(ecc, orc, gpu, fmt):
    """Decoding in pieces with the carry state == decoding the whole buffer."""
    ev = concat(events_random(80_000, 31, t_span=1 << 27), events_rows(4000, 32))
    words = orc.evt_encode(fmt, *ev, seed=9, noise_pct=10)
    rng = np.random.default_rng(4)
    cuts = np.sort(rng.choice(np.arange(1, len(words)), 40, replace=False))
    cuts = np.unique(np.concatenate([cuts, [cuts[0] + 1, 4096, 4097, 8192, 8193]]))  # incl. 1-word pieces
    got = _gpu_decode(ecc, gpu, fmt, words, pieces=cuts)
    _check_same(got, orc.evt_decode(fmt, words))


@pytest.mark.gpu
def test_gpu_evt_capacity(ecc, orc, gpu):
    ev = events_random(50_000, 41)
    words = orc.evt_encode(3, *ev, seed=2)
    ref = orc.evt_decode(3, words)
    got = _gpu_decode(ecc, gpu, 3, words, cap=12_345)
    assert got[3] == len(ref[0]) and got[4] == ecc.ERR_CAPACITY
    assert (got[0] == ref[0][:12_345]).all() and (got[1] == ref[1][:12_345]).all()


@pytest.mark.gpu
def test_gpu_evt_full_size_roundtrip(ecc, orc, gpu):
    """BASELINE C4 size: 20 M events through encode -> GPU decode == the original stream."""
    n = 20_000_000
    xy, t, p = ecc.gen_events(n, seed=1, width=346, height=260)
    for fmt in (3, 2):
        words = orc.evt_encode(fmt, xy, t, p, seed=1, noise_pct=2)
        got = _gpu_decode(ecc, gpu, fmt, words)
        assert got[3] == n
        _check_same(got, (xy, t, p))


@pytest.mark.gpu
def test_gpu_reslice_matches_oracle(ecc, orc, gpu):
    rng = np.random.default_rng(5)
    t = np.sort(rng.integers(-50_000, 3_000_000, 400_000)).astype(np.int64)
    t = np.concatenate([t, [9_000_000, 9_000_000, 9_000_001]])  # gap: empty slices
    d_t = ecc.DeviceArray.from_numpy(t)
    for period, max_slices in [(50_000, 1000), (1, 10_000_000), (777, 5)]:
        ref, ns = orc.reslice_n_us(t, period, max_slices)
        d_b = ecc.DeviceArray(max_slices + 1, np.int64)
        d_ns = ecc.DeviceArray(1, np.int64)
        gpu.reslice_n_us(d_t, len(t), period, d_b, max_slices, d_ns)
        st = gpu.evt_status()
        assert int(d_ns.numpy()[0]) == ns
        m = min(ns, max_slices)
        assert (d_b.numpy()[:m + 1] == ref[:m + 1]).all()
        assert st == (ecc.ERR_CAPACITY if ns > max_slices else 0)
    bad = ecc.DeviceArray.from_numpy(np.array([5, 4, 6], np.int64))
    d_b = ecc.DeviceArray(10, np.int64)
    d_ns = ecc.DeviceArray(1, np.int64)
    gpu.reslice_n_us(bad, 3, 2, d_b, 9, d_ns)
    assert gpu.evt_status() == ecc.ERR_UNSORTED_TIME


@pytest.mark.gpu
def test_gpu_raw_file_to_corners(ecc, orc, gpu, tmp_path):
    """A RAW recording on disk -> host reader -> GPU decode == the events that were written."""
    xy, t, p = ecc.gen_events(500_000, seed=3, width=346, height=260)
    words = orc.evt_encode(3, xy, t, p, seed=4)
    path = tmp_path / "rec.raw"
    path.write_bytes(b"% evt 3.0\n% format EVT3;height=260;width=346\n% end\n" + words.tobytes())
    info = ecc.raw_probe(path)
    w = ecc.raw_read_words(path, info)
    got = _gpu_decode(ecc, gpu, info.format, w)
    _check_same(got, (xy, t, p))


@pytest.mark.parametrize("fmt", [2, 3])
def test_raw_writer_roundtrip(ecc, orc, fmt):
    """Product RAW writer (ecc_evt_encode) -> oracle decoder == the events (incl. loops, rows)."""
    ev = concat(events_random(20_000, 51, t_span=1 << 27), events_rows(2000, 52))
    words = ecc.evt_encode(fmt, *ev)
    _check_same(orc.evt_decode(fmt, words), ev)
    if fmt == 3:
        assert ((words >> 12) == 4).sum() > 200
    with pytest.raises(ecc.EccError):
        ecc.evt_encode(fmt, ev[0][:3], np.array([5, 4, 6], np.int64), ev[2][:3])
