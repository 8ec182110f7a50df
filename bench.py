#!/usr/bin/env python3
"""Benchmark: end-to-end event pipeline throughput on MI355X (BASELINE.json metric
"Mevents/s (downsample+cluster+corner)").

One step = one pass of the hot path over one resident batch of synthetic events:
  hash downsample (8192-event windows)  ->  k-means k=16 on the representatives (10 Lloyd
  iterations + final labels), and SAE + FAST/arc corner detection (16384-event slices)  ->
  greedy 15x15 box NMS per slice.  On one GPU the two chains run on two HIP streams.
The corner tracker (sequential over slices) is timed separately and reported in µs/slice.

Single GPU:  python bench.py [--steps K --warmup W]
Multi GPU:   python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
  Each rank owns one contiguous time window (shard) of the stream: downsample and detection are
  shard-local; k-means is global from ONE RCCL all-reduce of the shards' per-pixel count images
  (every rank then runs the Lloyd passes locally); the SAE is handed over exactly (all-gather
  of the shards' own last-timestamp images; rank r starts from the elementwise max over ranks
  < r).  Weak scaling: events per rank fixed.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "event-camera-clustering-and-optical-flow-estimation_amd"
sys.path.insert(0, str(PKG))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--events", type=int, default=1221 * 16384,
                    help="events per GPU per step (1221 slices of 16384 = 20.0 M, BASELINE C4)")
    ap.add_argument("--width", type=int, default=346)
    ap.add_argument("--height", type=int, default=260)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cpu-events", type=int, default=40_000_000,
                    help="CPU-baseline sample size (~16 s of single-thread oracle work)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-tracker", action="store_true")
    ap.add_argument("--no-ingest", action="store_true", help="skip the RAW (EVT 3.0 / 2.0) decode measurement")
    ap.add_argument("--no-eps", action="store_true", help="skip the eps-neighbourhood (DBSCAN / OPTICS) measurement")
    ap.add_argument("--serial", action="store_true",
                    help="one stream for the whole step (isolated per-kernel times for profiling)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the single-GPU step as a captured HIP graph (measured equal to eager)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) on GPUs; gloo for rehearsal")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on device 0 (with --dist-backend gloo)")
    return ap.parse_args()


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        local = 0
    dist = None
    torch = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group(args.dist_backend)
        dist = tdist
    import eccpy as ecc

    W, H, n, K, I = args.width, args.height, args.events, args.k, args.iters
    if n % 16384:
        raise SystemExit("--events must be a multiple of the 16384-event slice (global slice alignment)")
    # one stream for libecc and the collectives (torch's current stream) when sharded
    ctx = ecc.Context(local, stream=torch.cuda.current_stream().cuda_stream) if dist else ecc.Context(local)
    xy_h, t_h, p_h = ecc.gen_events(n, first=rank * n, seed=1, width=W, height=H)
    d_xy, d_t = ecc.DeviceArray.from_numpy(xy_h, ctx.stream), ecc.DeviceArray.from_numpy(t_h, ctx.stream)
    hcfg = ecc.hash_cfg(window=8192)  # reference bounds 0<=x<=1280, 0<=y<=720
    n_win = (n + 8191) // 8192
    rep_xy = ecc.DeviceArray(n_win * 8192, np.uint32)
    uniq = ecc.DeviceArray(n_win, np.int32)
    rep = ecc.DeviceArray(n_win, np.int32)
    c0 = np.stack([np.linspace(20, W - 20, K), np.linspace(20, H - 20, K)[::-1]], 1).astype(np.float32).ravel()
    d_c0 = ecc.DeviceArray.from_numpy(c0, ctx.stream)
    d_c = ecc.DeviceArray(2 * K, np.float32)
    labels = ecc.DeviceArray(n_win * 8192, np.uint8)
    kcfg = ecc.kmeans_cfg(k=K, max_iters=I, tol=-1.0)
    ccfg = ecc.corner_cfg(width=W, height=H, first_detect_slice=1 if rank == 0 else 0)
    sae = ecc.DeviceArray(W * H, np.int64)
    flags = ecc.DeviceArray(n, np.uint8)
    ns, cap = (n + 16383) // 16384, 4096
    nms_out = ecc.DeviceArray(ns * cap, ecc.CORNER_DTYPE)
    nms_cnt = ecc.DeviceArray(ns, np.int32)
    lib = ecc.lib
    if dist:
        # exchange buffers are torch tensors (RCCL operates on them); libecc gets their pointers
        t_counts = torch.zeros(W * H, dtype=torch.int32, device=f"cuda:{local}")
        t_local = torch.zeros(W * H, dtype=torch.int64, device=f"cuda:{local}")
        t_all = torch.zeros(world * W * H, dtype=torch.int64, device=f"cuda:{local}")

    def step_sharded():
        """Shard-local downsample/detection/NMS; global k-means from ONE all-reduce of the
        shards' per-pixel count images; exact SAE hand-off (all-gather of the shards' own last-t
        images, computed by the detection's prepare phase)."""
        S = ctx.stream
        ecc.check(lib.ecc_downsample_hash(ctx.ctx, d_xy.ptr, n, ecc.C.byref(hcfg), rep_xy.ptr, None,
                                          uniq.ptr, rep.ptr, S), "downsample")
        ecc.check(lib.ecc_kmeans_counts_xy16(ctx.ctx, rep_xy.ptr, n_win, 8192, uniq.ptr, W, H, t_counts.data_ptr(), S))
        ecc.check(lib.ecc_fast_detect_prepare(ctx.ctx, d_xy.ptr, d_t.ptr, n, ecc.C.byref(ccfg), t_local.data_ptr(), S))
        dist.all_reduce(t_counts)
        dist.all_gather_into_tensor(t_all, t_local)
        ecc.check(lib.ecc_memcpy_d2d(d_c.ptr, d_c0.ptr, 8 * K, S))
        ecc.check(lib.ecc_kmeans_run_counts(ctx.ctx, t_counts.data_ptr(), W, H, ecc.C.byref(kcfg), d_c.ptr, None, S))
        ecc.check(lib.ecc_kmeans_labels_xy16(ctx.ctx, rep_xy.ptr, n_win, 8192, uniq.ptr, d_c.ptr, K,
                                             kcfg.threshold, labels.ptr, S))
        ecc.check(lib.ecc_sae_max_combine(ctx.ctx, t_all.data_ptr(), rank, W * H, sae.ptr, S))
        ecc.check(lib.ecc_fast_detect_finish(ctx.ctx, d_xy.ptr, d_t.ptr, n, ecc.C.byref(ccfg), sae.ptr,
                                             flags.ptr, S), "fast_detect_finish")
        ctx.corner_nms(d_xy, flags, n, 16384, W, H, 15, cap, nms_out, nms_cnt)

    # single GPU: downsample -> k-means and the corner chain read the same resident batch and are
    # independent, so they run on two streams (fork/join with events) and overlap
    s2, ev_fork, ev_join = ecc.P(), ecc.P(), ecc.P()
    if not dist:
        ecc.check(lib.ecc_stream_create(ecc.C.byref(s2)), "stream")
        ecc.check(lib.ecc_event_create(ecc.C.byref(ev_fork)), "event")
        ecc.check(lib.ecc_event_create(ecc.C.byref(ev_join)), "event")

    def step(serial=args.serial):
        if dist:
            return step_sharded()
        ks = ctx.stream if serial else s2.value  # the k-means chain's stream
        ecc.check(lib.ecc_event_record(ev_fork, ctx.stream))
        ecc.check(lib.ecc_stream_wait_event(ks, ev_fork))
        ecc.check(lib.ecc_downsample_hash(ctx.ctx, d_xy.ptr, n, ecc.C.byref(hcfg), rep_xy.ptr, None,
                                          uniq.ptr, rep.ptr, ks), "downsample")
        ecc.check(lib.ecc_memcpy_d2d(d_c.ptr, d_c0.ptr, 8 * K, ks))
        ecc.check(lib.ecc_kmeans_run_xy16(ctx.ctx, rep_xy.ptr, n_win, 8192, uniq.ptr, ecc.C.byref(kcfg), d_c.ptr,
                                          labels.ptr, None, ks), "kmeans")
        ecc.check(lib.ecc_event_record(ev_join, ks))
        ecc.check(lib.ecc_memset_async(sae.ptr, 0, sae.nbytes, ctx.stream))
        ctx.fast_detect(d_xy, d_t, n, ccfg, sae, flags)
        ctx.corner_nms(d_xy, flags, n, 16384, W, H, 15, cap, nms_out, nms_cnt)
        ecc.check(lib.ecc_stream_wait_event(ctx.stream, ev_join))

    for _ in range(args.warmup):
        step()
    ctx.sync()
    if ctx.fast_detect_status() != 0:
        raise RuntimeError("fast_detect reported a status error")
    if dist and lib.ecc_kmeans_counts_status(ctx.ctx, ctx.stream) != 0:
        raise RuntimeError("a representative lies outside the k-means count frame")
    n_reps = int(uniq.numpy().sum())
    # --graph: the step's ~40 launches and memsets are captured once into a HIP graph
    # (ecc_graph_*) and replayed — the same kernels on the same buffers, without per-launch
    # host dispatch (measured equal to eager: the GPU is the bottleneck).  The sharded step
    # interleaves RCCL collectives and stays eager.
    graph = None
    if not dist and args.graph:
        gp = ecc.P()
        ecc.check(lib.ecc_graph_begin(ctx.stream), "ecc_graph_begin")
        step()
        ecc.check(lib.ecc_graph_end(ctx.stream, ecc.C.byref(gp)), "ecc_graph_end")
        graph = gp.value
        ecc.check(lib.ecc_graph_launch(graph, ctx.stream), "ecc_graph_launch")  # one untimed replay
        ctx.sync()

    def timed_step():
        if graph is not None:
            ecc.check(lib.ecc_graph_launch(graph, ctx.stream), "ecc_graph_launch")
        else:
            step()

    # 1. the timed region: K steps, uninstrumented (a timestamped HIP event around every launch
    #    drains the queue between kernels and costs ~0.6 ms/step here)
    if dist:
        dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        timed_step()
    ctx.sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # 2. the kernel-timing pass: the same K steps again with HIP events recorded around every
    #    launch on its stream (ecc_ctx_set_timing) -> per-kernel average durations.  It runs on
    #    ONE stream, so that a kernel's time is its own (not queueing behind the other chain).
    lib.ecc_ctx_set_timing(ctx.ctx, 1)
    lib.ecc_ctx_timing_reset(ctx.ctx)
    ctx.sync()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step(serial=True)
    ctx.sync()
    instrumented = time.perf_counter() - t1
    lib.ecc_ctx_set_timing(ctx.ctx, 0)
    buf = ecc.C.create_string_buffer(1 << 16)
    ecc.check(lib.ecc_ctx_timing_report(ctx.ctx, buf, len(buf)))
    stats = json.loads(buf.value.decode())

    # per-kernel roofline of the dominant kernel (largest total time in the timed region)
    kern_ms = {k: v["total_ms"] for k, v in stats.items()}
    dominant = max(kern_ms, key=kern_ms.get)
    launches = stats[dominant]["launches"]
    avg_ms = kern_ms[dominant] / launches
    per_step_launches = launches / args.steps
    # algorithmic bytes per launch: what the kernel must move at minimum
    geo = corner_geometry(xy_h, n, W, H)
    bytes_per_launch = {
        "downsample_hash_kernel": 4.0 * n + 4.0 * n_reps + 8.0 * n_win,   # xy in, reps + counts out
        "kmeans_xy16_kernel": 4.0 * n_reps,                               # packed u16 xy per point
        "kmeans_xy16_labels": 5.0 * n_reps,                               # + u8 label out
        "kmeans_count_kernel": 4.0 * n_reps,                              # packed u16 xy per point
        "kmeans_pixel_pass": 4.0 * W * H,                                 # per-pixel counts (bbox <= sensor)
        # corner stage: xy + t in, key + t32 out (+ per-slice tile offsets)
        "slice_sort_kernel": 20.0 * n + 4.0 * geo["slices"] * (geo["tiles"] + 2),
        # key + t32 in, pair entries out, per-(group, pixel) slice mask + last t out
        "pair_build_kernel": 8.0 * n + 8.0 * geo["pairs"] + 12.0 * geo["hw_groups"],
        # each pair entry read once, B_g per (group, pixel), corner-pair bits out
        "arc_kernel": 8.0 * geo["pairs"] + 8.0 * geo["hw_groups"] + 784.0 * geo["items"],
        "flags_kernel": 5.0 * n,                                          # xy in, flags out
        "sae_prefix_kernel": 20.0 * geo["hw_groups"] + 16.0 * W * H,
        "nms_kernel": 1.0 * n,                                            # corner flags
    }.get(dominant, 0.0)
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    # HBM bytes per launch of the same kernel from the newest committed PMC summary
    # (scripts/gpu_profile.sh + scripts/traffic.py; PMC passes cannot run inside this process)
    traffic = None
    tfiles = sorted((ROOT / "profiles").glob("*_traffic.json"))
    if tfiles:
        try:
            rec = json.loads(tfiles[-1].read_text()).get(dominant)
            traffic = round(rec["bytes_per_launch"]) if rec else None
        except (ValueError, KeyError, TypeError):
            traffic = None

    # tracker (sequential over slices): reported separately, µs per slice
    tracker_us = None
    if not args.no_tracker and rank == 0:
        tr = ecc.Tracker(ctx)
        tmr = ecc.Timer(ctx.stream)
        tmr.start()
        tr.update(nms_out, nms_cnt, ns, cap)
        tracker_us = tmr.stop() * 1e3 / ns
        tr.close()

    # RAW ingest, reported beside the headline: the same events written
    # as EVT 3.0 / EVT 2.0 words, decoded from device-resident words.
    ingest = None
    if not args.no_ingest and rank == 0:
        ingest = {}
        for fmt, name in ((ecc.EVT3, "EVT3"), (ecc.EVT2, "EVT2")):
            words = ecc.evt_encode(fmt, xy_h, t_h, p_h)
            d_words = ecc.DeviceArray.from_numpy(words, ctx.stream)
            d_oxy, d_ot = ecc.DeviceArray(n, np.uint32), ecc.DeviceArray(n, np.int64)
            d_op, d_on = ecc.DeviceArray(n, np.uint8), ecc.DeviceArray(1, np.int64)
            run = lambda: ctx.evt_decode(fmt, d_words, len(words), d_oxy, d_ot, d_op, n, d_on)
            run()
            ctx.sync()
            reps = max(args.steps, 5)
            tmr = ecc.Timer(ctx.stream)
            tmr.start()
            for _ in range(reps):
                run()
            dec_ms = tmr.stop() / reps
            assert int(d_on.numpy()[0]) == n and ctx.evt_status() == 0
            ctx.set_timing(True)
            ctx.timing_reset()
            for _ in range(reps):
                run()
            st = ctx.timing_report()
            ctx.set_timing(False)
            kern = {k: v["total_ms"] / v["launches"] for k, v in st.items()}
            wbytes = words.nbytes
            dk = kern.get("evt_decode_kernel", float("nan"))
            ach = (wbytes + 13.0 * n) / (dk * 1e-3) / 1e9  # words in + xy/t/p out
            ingest[name] = {
                "words": len(words), "word_bytes": words.itemsize, "events": n,
                "mevents_s": round(n / (dec_ms * 1e-3) / 1e6, 1), "ms_per_decode": round(dec_ms, 4),
                "kernels_us": {k: round(v * 1e3, 2) for k, v in sorted(kern.items())},
                "roofline": {"kernel": "evt_decode_kernel", "bound": "hbm", "achieved": round(ach, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                             "algorithmic_bytes": f"{words.itemsize} B/word in + 13 B/event out"},
            }
            del d_words, d_oxy, d_ot, d_op, d_on

    # eps-neighbourhoods (BASELINE C4), reported beside the headline:
    # DBSCAN eps 20 / minPts 20 (counts) and OPTICS eps 10 / min_pts 2 (counts + core distances)
    # per 8192-event downsample window, over this step's device-resident representatives.
    eps_res = None
    if not args.no_eps and rank == 0:
        eps_res = {}
        e_cnt = ecc.DeviceArray(n_win * 8192, np.int32)
        e_core = ecc.DeviceArray(n_win * 8192, np.float64)
        for name, eps, mp, core in (("dbscan_eps20_minpts20", 20.0, 20, None),
                                    ("optics_eps10_minpts2", 10.0, 2, e_core)):
            run = lambda: ctx.eps_counts(rep_xy, n_win, 8192, uniq, eps, mp, e_cnt, core)
            run()
            ctx.sync()
            reps = max(args.steps, 5)
            tmr = ecc.Timer(ctx.stream)
            tmr.start()
            for _ in range(reps):
                run()
            call_ms = tmr.stop() / reps
            ctx.set_timing(True)
            ctx.timing_reset()
            for _ in range(reps):
                run()
            st = ctx.timing_report()
            ctx.set_timing(False)
            kern = {k: v["total_ms"] / v["launches"] for k, v in st.items()}
            ek = kern.get("eps_counts_kernel", float("nan"))
            per_rep = 8 + (8 if core is not None else 0)  # xy in + count out [+ core distance out]
            ach = n_reps * per_rep / (ek * 1e-3) / 1e9
            eps_res[name] = {
                "reps": n_reps, "windows": n_win, "mreps_s": round(n_reps / (call_ms * 1e-3) / 1e6, 1),
                "ms_per_call": round(call_ms, 4), "kernels_us": {k: round(v * 1e3, 2) for k, v in sorted(kern.items())},
                "roofline": {"kernel": "eps_counts_kernel", "bound": "hbm", "achieved": round(ach, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                             "algorithmic_bytes": f"4 B/rep in + 4 B/rep out{' + 8 B/rep core distance' if core is not None else ''}"},
            }
        del e_cnt, e_core

    value = world * args.steps * n / elapsed / 1e6
    if graph is not None:
        lib.ecc_graph_destroy(graph)
    result = {
        "metric": "Mevents/s (downsample+cluster+corner)",
        "value": round(value, 2),
        "unit": "Mevents/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16xy/i64t (int), fp32 k-means",
        "data": "synthetic (seeded splitmix64 event generator: moving polygons + Gaussian blobs + noise)",
        "config": {
            "workload": f"e2e hash-downsample(8192-event windows) -> k-means k={K} ({I} iters) on reps -> "
                        f"SAE+FAST arc corners (16384-event slices) -> 15x15 NMS; {W}x{H} sensor; "
                        f"{n} events/GPU/step (BASELINE configs C2-C4)",
            "events_per_gpu": n, "reps_per_gpu": n_reps, "width": W, "height": H, "k": K,
            "kmeans_iters": I, "parallelism": f"time-window shards x{world}",
            "launch": "hipGraph replay of the captured step" if graph is not None else "eager launches",
        },
        "roofline": {
            "kernel": dominant, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "avg_launch_ms": round(avg_ms, 5), "algorithmic_bytes_per_launch": bytes_per_launch,
            "timing": f"HIP events around every launch in a second, eager, one-stream {args.steps}-step "
                      f"pass ({instrumented / args.steps * 1e3:.3f} ms/step instrumented)",
        },
        "stages_ms_per_step": {k: round(v / args.steps, 4) for k, v in sorted(kern_ms.items())},
        "tracker_us_per_slice": None if tracker_us is None else round(tracker_us, 2),
        "ingest": ingest,
        "eps": eps_res,
    }
    if rank == 0 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args, W, H, K, I)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def corner_geometry(xy, n, W, H, S=16384, group=32, tile=14):
    """Counts the corner stage's byte table needs: distinct (slice, pixel) pairs of in-sensor
    events (= pair entries), (group, tile) items, (group, pixel) image cells."""
    x = (xy & 0xFFFF).astype(np.int64)
    y = (xy >> 16).astype(np.int64)
    inside = (x < W) & (y < H)
    s = np.arange(n, dtype=np.int64) // S
    pairs = int(np.unique((s * (W * H) + y * W + x)[inside]).size)
    slices = (n + S - 1) // S
    groups = (slices + group - 1) // group
    tiles = ((W + tile - 1) // tile) * ((H + tile - 1) // tile)
    return {"pairs": pairs, "slices": slices, "tiles": tiles, "items": groups * tiles, "hw_groups": groups * W * H}


def cpu_baseline(args, W, H, K, I):
    """The oracle (single-thread -O2 C++ restatement of the reference algorithms) on the first
    `--cpu-events` events of the same stream, on this host's cores."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import eccpy as ecc
    import orc

    m = args.cpu_events
    xy, t, _ = ecc.gen_events(m, seed=1, width=W, height=H)
    c0 = np.stack([np.linspace(20, W - 20, K), np.linspace(20, H - 20, K)[::-1]], 1).astype(np.float32).ravel()
    t0 = time.perf_counter()
    rx, _, u, _ = orc.downsample_hash(xy)
    dense = np.concatenate([rx[w * 8192: w * 8192 + u[w]] for w in range(len(u))])
    orc.kmeans_run_xy16(dense, c0, I)
    fl, _ = orc.fast_detect(xy, t, W, H)
    orc.corner_nms(xy, fl, W, H)
    dt = time.perf_counter() - t0
    model = ""
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = platform.processor()
    return {"value": round(m / dt / 1e6, 3), "unit": "Mevents/s", "cores": 1, "kind": "port",
            "sample": f"first {m} events of the same stream, same pipeline (oracle/oracle.cpp, 1 thread); "
                      f"{dt:.2f} s; host {model}, nproc={os.cpu_count()}"}


if __name__ == "__main__":
    main()
