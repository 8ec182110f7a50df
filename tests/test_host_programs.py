"""The C++ host layer (include/ecc.hpp) and the host programs mirroring the reference mains,
run on the GPU and checked against the oracle / the reference's KATs."""
import json
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "event-camera-clustering-and-optical-flow-estimation_amd" / "bin"
GOLDEN = ROOT / "tests" / "golden"


def run(prog, *args):
    r = subprocess.run([str(BIN / prog)] + [str(a) for a in args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def parse_order(out):
    line = [l for l in out.splitlines() if l.startswith("order")][0]
    pairs = [p.split(":") for p in line.split()[1:]]
    return np.array([int(a) for a, _ in pairs]), np.array([float(b) for _, b in pairs])


@pytest.mark.parametrize("name", ["clustering_test_1", "clustering_test_2"])
def test_optics_kat_through_cpp_api(tmp_path, name):
    kat = json.loads((GOLDEN / "optics_kat.json").read_text())[name]
    f = tmp_path / "pts.csv"
    f.write_text("\n".join(f"{x},{y}" for x, y in kat["points"]) + "\n")
    out = run("ecc_optics_events", "--points", f, "--min-pts", kat["min_pts"], "--eps", kat["eps"],
              "--threshold", kat["threshold"])
    order, reach = parse_order(out)
    clusters, cur = [], None
    for i, r in zip(order, reach):
        if r < 0 or r >= kat["threshold"] or cur is None:
            cur = [int(i)]
            clusters.append(cur)
        else:
            cur.append(int(i))
    assert [sorted(c) for c in clusters] == kat["clusters"]


def test_optics_event_fixture_matches_oracle(orc, ecc):
    out = run("ecc_optics_events", GOLDEN / "event_raw_data8.csv")
    order, reach = parse_order(out)
    xy, _, _ = ecc.read_csv(GOLDEN / "event_raw_data8.csv")
    x, y = ecc.unpack_xy(xy)
    o_order, o_reach = orc.optics(np.stack([x, y], 1).astype(np.float64), 2, 10.0)
    assert (order == o_order).all()
    assert np.array_equal(reach, o_reach)


def test_optics_large_window_matches_oracle(orc, ecc, tmp_path):
    """N = 9548 as in cluster_event_data.cpp:332 (> one 8192 window)."""
    xy, _, _ = ecc.gen_events(30000, seed=12)
    rx, _, u, _ = orc.downsample_hash(xy, window=16384)
    pts = rx[:u[0]]
    x, y = ecc.unpack_xy(pts)
    f = tmp_path / "p.csv"
    f.write_text("\n".join(f"{a},{b}" for a, b in zip(x, y)) + "\n")
    out = run("ecc_optics_events", "--points", f)
    order, reach = parse_order(out)
    o_order, o_reach = orc.optics(np.stack([x, y], 1).astype(np.float64), 2, 10.0)
    assert len(order) == len(x) and (order == o_order).all() and np.array_equal(reach, o_reach)


def test_kmeans_demo_matches_oracle(orc):
    out = run("ecc_kmeans_demo")
    vals = [tuple(map(float, m)) for m in re.findall(r"\(([-\d.]+), ([-\d.]+), (\d+)\)", out)]
    data = (np.arange(4096) % 100).astype(np.float32)
    c0 = np.array([1, 1, 10, 10, 20, 20, 30, 30, 50, 50, 60, 60, 70, 70, 80, 80], np.float32)
    o_c, o_lab, _ = orc.kmeans_run_f32(data, c0, 20, 50.0, 10.0)
    g = np.array([[a, b] for a, b, _ in vals], np.float32).ravel()
    assert np.allclose(g, o_c, atol=1e-4)
    assert [int(c) for _, _, c in vals] == [int((o_lab == j).sum()) for j in range(8)]


def test_corner_track_program_matches_oracle(orc, ecc):
    n, W, H = 16384 * 20, 346, 260
    out = run("ecc_corner_track", "--synthetic", n, "--width", W, "--height", H)
    xy, t, _ = ecc.gen_events(n, width=W, height=H)
    flags, _ = orc.fast_detect(xy, t, W, H)
    o_out, o_cnt, _ = orc.corner_nms(xy, flags, W, H)
    rows = re.findall(r"Corner size : (\d+)  Filtered corner size : (\d+)", out)
    assert [int(a) for a, _ in rows] == [int(flags[s * 16384:(s + 1) * 16384].sum()) for s in range(20)]
    assert [int(b) for _, b in rows] == list(o_cnt)
    tr = orc.OracleTracker(ecc.tracker_cfg())
    for s in range(20):
        tr.update(o_out[s * 4096: s * 4096 + o_cnt[s]])
    exp = [(t.label, t.x, t.y, t.frame_count) for t in tr.tracks(ecc.Track)]
    got = [tuple(map(int, m)) for m in re.findall(r"track label (\d+) pos \((\d+),(\d+)\) frames (\d+)", out)]
    assert got == exp


def test_downsample_program_matches_oracle(orc, ecc):
    out = run("ecc_downsample_store", "--synthetic", 100000)
    xy, _, _ = ecc.gen_events(100000, width=1280, height=720)  # the program's sensor
    _, _, u, r = orc.downsample_hash(xy)
    got = [tuple(map(int, m)) for m in re.findall(r"unique_count: (\d+), repeated_count: (\d+)", out)]
    assert got == list(zip(u.tolist(), r.tolist()))


def test_dbscan_program_matches_oracle(orc, ecc, tmp_path):
    xy, t, _ = ecc.gen_events(8192, seed=5)
    rx, _, u, _ = orc.downsample_hash(xy)
    pts = rx[:u[0]]
    x, y = ecc.unpack_xy(pts)
    f = tmp_path / "e.csv"
    f.write_text("\n".join(f"{a},{b},0,0" for a, b in zip(x, y)) + "\n")
    out = run("ecc_dbscan", f, "--eps", 10, "--min-pts", 8, "--min-size", 20)
    k = int(re.search(r"cluster size : (\d+)", out).group(1))
    pts3 = np.stack([x, y, np.zeros_like(x)], 1).astype(np.float32)
    ok, olab = orc.dbscan(pts3, 10.0, 8, 20, 25000)
    assert k == ok and k > 0
    lines = [l.split(",") for l in out.splitlines()[1:] if l.count(",") == 3]
    # membership per point position: (x,y) -> cluster id % 8
    got = {(int(float(a)), int(float(b))): int(c) for a, b, _, c in lines}
    for i in range(len(x)):
        if olab[i] >= 0:
            assert got[(int(x[i]), int(y[i]))] == olab[i] % 8


@pytest.mark.parametrize("fmt", [3, 2])
def test_corner_track_program_reads_raw_recording(orc, ecc, tmp_path, fmt):
    """argv[1] = a RAW recording (Camera::from_file, FCT/…group_track.cpp:756-760): the program's
    output equals its output on the same events given as --synthetic."""
    n, W, H = 16384 * 12, 346, 260
    xy, t, p = ecc.gen_events(n, width=W, height=H)
    words = orc.evt_encode(fmt, xy, t, p, seed=2)
    path = tmp_path / "rec.raw"
    hdr = f"% evt {fmt}.0\n% geometry {W}x{H}\n% end\n"
    path.write_bytes(hdr.encode() + words.tobytes())
    a = run("ecc_corner_track", path, "--width", W, "--height", H)
    b = run("ecc_corner_track", "--synthetic", n, "--width", W, "--height", H)
    assert a == b and "Corner size" in a


def _parse_cluster_program(out):
    windows, rows = [], []
    w = -1
    for line in out.splitlines():
        m = re.match(r"window (\d+) reps (\d+) clusters (\d+)", line)
        if m:
            w = int(m.group(1))
            windows.append(int(m.group(3)))
            continue
        m = re.match(r"\s+cluster (\d+) n (\d+) centroid (\S+) (\S+) flow (.*)", line)
        if m:
            fl = m.group(5).split()
            rows.append([w, int(m.group(1)), int(m.group(2)), float(m.group(3)), float(m.group(4)),
                         0.0 if fl == ["-"] else 1.0,
                         *([float("nan")] * 2 if fl == ["-"] else [float(fl[0]), float(fl[1])])])
    return windows, np.array(rows, np.float64).reshape(-1, 8)


@pytest.mark.parametrize("args,kw", [
    ((), {}),                                                  # the reference's defaults (AEClustering.cpp:7-18)
    (("--kappa", 100000), {"kappa": 100000}),                  # sampled distance = full scan (kappa > n)
    (("--radius", 10, "--min-n", 3), {"radius": 10.0, "min_n": 3}),
])
def test_downsample_cluster_program_matches_oracle(orc, ecc, tmp_path, args, kw):
    """GPU downsample -> AEClustering -> centroid flow (DSA/…opencl_store.cpp:370-518) vs the oracle."""
    n, W, H = 8192 * 40, 346, 260
    out = run("ecc_downsample_cluster", "--synthetic", n, "--width", W, "--height", H, *args,
              "--ppm-dir", tmp_path, "--csv", tmp_path / "c.csv")
    xy, _, _ = ecc.gen_events(n, width=W, height=H)
    rx, _, u, _ = orc.downsample_hash(xy)
    o_rows, o_cpw = orc.aec_run(rx, u, **kw)
    windows, rows = _parse_cluster_program(out)
    assert windows == list(o_cpw)
    assert rows.shape == o_rows.shape and rows.shape[0] > 0
    assert np.array_equal(rows[:, :6], o_rows[:, :6])
    has = o_rows[:, 5] == 1
    assert np.array_equal(rows[has, 6:], o_rows[has, 6:])
    ppm = (tmp_path / "cluster_frame_combined1.ppm").read_bytes()
    assert ppm.startswith(f"P6\n{W} {H}\n255\n".encode()) and len(ppm) == len(f"P6\n{W} {H}\n255\n") + W * H * 3
    assert (tmp_path / "c.csv").stat().st_size > 0
