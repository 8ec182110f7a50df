#!/usr/bin/env python3
"""Benchmark: end-to-end event pipeline throughput on MI355X (BASELINE.json metric
"Mevents/s (downsample+cluster+corner)").

One step = one pass of the hot path over one resident batch of synthetic events:
  hash downsample (8192-event windows)  ->  k-means k=16 on the representatives (10 Lloyd
  iterations + final labels), and SAE + FAST/arc corner detection (16384-event slices)  ->
  greedy 15x15 box NMS per slice.  On one GPU the two chains run on two HIP streams.
The corner tracker (sequential over slices) is outside the metric's stages; it is measured
beside it: µs per slice, and the pipelined throughput with the tracker of batch b running on a
third stream while batch b+1 is detected (`with_tracker`).

Single GPU:  python bench.py [--steps K --warmup W]
Multi GPU:   python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
  Each rank owns one contiguous time window (shard) of the stream: downsample and detection are
  shard-local; k-means is global from ONE RCCL all-reduce of the shards' per-pixel count images
  (every rank then runs the Lloyd passes locally); the SAE is handed over exactly (all-gather
  of the shards' own last-timestamp images; rank r starts from the elementwise max over ranks
  < r).  After the timed steps the shards' NMS lists are gathered in global slice order and ONE
  tracker on rank 0 consumes them (the C5 track merge, `track_merge`).  Weak scaling: events per
  rank fixed (--events; --preset c5 = 50 M per GPU, BASELINE config C5).
Rank 0 prints ONE JSON line.  With the CPU leg on (default, rank 0 of a 1-GPU run), the oracle
runs the same pipeline over exactly the step's events: that is the CPU baseline, and every GPU
output of the step is compared with it (`parity`).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "event-camera-clustering-and-optical-flow-estimation_amd"
sys.path.insert(0, str(PKG))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SLICE = 16384
WINDOW = 8192
CORNER_KERNELS = ("slice_sort_kernel", "pair_build_kernel", "sae_prefix_kernel", "arc_kernel",
                  "arc_dense_kernel", "flags_kernel")
KMEANS_KERNELS = ("kmeans_count_kernel", "kmeans_count_sum_kernel", "kmeans_extent_kernel",
                  "kmeans_pixel_pass", "kmeans_step_kernel", "kmeans_xy16_labels")
NMS_KERNELS = ("nms_compact_kernel", "nms_kernel")


PRESET_SLICES = {"c4": 1221, "c5": 3052}  # 20 004 864 / 50 003 968 events per GPU


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--preset", choices=("c4", "c5"), default=None,
                    help="c4: 20.0 M events per GPU (1221 slices, BASELINE C4, the metric's config); "
                         "c5: 50.0 M events per GPU (3052 slices; 8 GPUs = the 400 M-event stream of C5). "
                         "Default: c4 on one GPU, c5 when --gpus > 1 (the multi-GPU line is BASELINE C5)")
    ap.add_argument("--events", type=int, default=None, help="events per GPU per step (overrides --preset)")
    ap.add_argument("--width", type=int, default=346)
    ap.add_argument("--height", type=int, default=260)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline and the full-size parity leg")
    ap.add_argument("--no-tracker", action="store_true")
    ap.add_argument("--no-ingest", action="store_true", help="skip the RAW (EVT 3.0 / 2.0) decode measurement")
    ap.add_argument("--no-eps", action="store_true", help="skip the eps-neighbourhood (DBSCAN / OPTICS) measurement")
    ap.add_argument("--no-c3", action="store_true", help="skip the BASELINE C3 k-means (k=16, 50 M points) measurement")
    ap.add_argument("--corner-shards", type=int, default=1,
                    help="one GPU: run the corner chain as this many time-window shards on their own contexts "
                         "and streams (the multi-GPU SAE hand-off inside the device)")
    ap.add_argument("--serial", action="store_true",
                    help="one stream for the whole step (isolated per-kernel times for profiling)")
    ap.add_argument("--joined", action="store_true",
                    help="one GPU: join the k-means stream at the end of every step (default: steps pipelined — "
                         "step i's k-means chain may still run beside step i+1's detection; r06k: 0.520 -> 0.50 ms)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the single-GPU step as a captured HIP graph (measured equal to eager)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) on GPUs; gloo for rehearsal")
    ap.add_argument("--dist-parity", action="store_true",
                    help="sharded runs: every rank recomputes the whole stream on the oracle and compares its "
                         "shard's outputs, the global centroids and (rank 0) the merged tracker (rehearsal sizes)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on device 0 (with --dist-backend gloo)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the sharded step even at world size 1: a 1-rank process group of --dist-backend "
                         "(nccl = RCCL), so the C5 code path — collectives, SAE combine, corner pack/gather, "
                         "track merge — executes on a single GPU")
    ap.add_argument("--overlap", action="store_true",
                    help="keep the two-stream sharded schedule under gloo too (correctness rehearsals; gloo "
                         "collectives block the host, so it is not a timing configuration)")
    ap.add_argument("--dist-native", action="store_true",
                    help="sharded runs: every device collective through libecc's own RCCL entry points "
                         "(ecc_dist_*: count all-reduce, SAE hand-off, corner gather); torch.distributed (gloo, "
                         "CPU) only carries the control plane (the RCCL unique id, barriers, the timing max)")
    ap.add_argument("--no-n1-rate", action="store_true",
                    help="sharded runs: skip rank 0's single-GPU rate at the same per-GPU size (per_gpu_rate_n1)")
    a = ap.parse_args(argv)
    if a.preset is None:
        a.preset = "c5" if a.gpus > 1 else "c4"
    if a.events is None:
        a.events = PRESET_SLICES[a.preset] * SLICE
    return a


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`--gpus N` without an external launcher: run N ranks of this script under
    `torch.distributed.run` as a CHILD process (nothing here has touched the GPU yet: no torch,
    no libecc, no exec) and return its exit code; rank 0 of the child prints the JSON line.
    Under a launcher (WORLD_SIZE set) the world size must equal --gpus."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != args.gpus and not (args.force_dist and args.gpus == 1 and int(world_env) == 1):
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env} (one rank per GPU: they must agree)",
                  file=sys.stderr, flush=True)
            return 2
        return None
    if args.gpus <= 1:
        return None
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["MASTER_ADDR"] = "127.0.0.1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(Path(__file__).resolve()),
           *sys.argv[1:]]
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        local = 0
    dist = None
    torch = None
    if world > 1 or args.force_dist:
        import torch
        import torch.distributed as tdist
        if world == 1:  # a 1-rank group needs its own rendezvous
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 2000))
        if not args.same_device and local >= torch.cuda.device_count():
            raise SystemExit(f"bench.py: rank {rank} needs device {local}, only {torch.cuda.device_count()} visible")
        torch.cuda.set_device(local)
        # --dist-native: the process group is the control plane only (gloo); the data path is
        # libecc's ecc_dist_* over RCCL
        tdist.init_process_group("gloo" if args.dist_native else args.dist_backend)
        dist = tdist
        if dist.get_world_size() != world:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")
    import eccpy as ecc

    W, H, n, K, I = args.width, args.height, args.events, args.k, args.iters
    if n % SLICE:
        raise SystemExit("--events must be a multiple of the 16384-event slice (global slice alignment)")
    # one stream for libecc and the collectives (torch's current stream) when sharded
    ctx = ecc.Context(local, stream=torch.cuda.current_stream().cuda_stream) if dist else ecc.Context(local)
    native = None
    if dist and args.dist_native:
        uid = [ecc.Dist.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        native = ecc.Dist(ctx, uid[0], world, rank)
    xy_h, t_h, p_h = ecc.gen_events(n, first=rank * n, seed=1, width=W, height=H)
    d_xy, d_t = ecc.DeviceArray.from_numpy(xy_h, ctx.stream), ecc.DeviceArray.from_numpy(t_h, ctx.stream)
    hcfg = ecc.hash_cfg(window=WINDOW)  # reference bounds 0<=x<=1280, 0<=y<=720
    n_win = (n + WINDOW - 1) // WINDOW
    rep_xy = ecc.DeviceArray(n_win * WINDOW, np.uint32)
    uniq = ecc.DeviceArray(n_win, np.int32)
    rep = ecc.DeviceArray(n_win, np.int32)
    c0 = np.stack([np.linspace(20, W - 20, K), np.linspace(20, H - 20, K)[::-1]], 1).astype(np.float32).ravel()
    d_c0 = ecc.DeviceArray.from_numpy(c0, ctx.stream)
    d_c = ecc.DeviceArray(2 * K, np.float32)
    labels = ecc.DeviceArray(n_win * WINDOW, np.uint8)
    kcfg = ecc.kmeans_cfg(k=K, max_iters=I, tol=-1.0)
    ccfg = ecc.corner_cfg(width=W, height=H, first_detect_slice=1 if rank == 0 else 0)
    sae = ecc.DeviceArray(W * H, np.int64)
    flags = ecc.DeviceArray(n, np.uint8)
    ns, cap = n // SLICE, 4096
    # two NMS output buffers: the pipelined tracker pass consumes batch b's while b+1 is detected
    nms_out = [ecc.DeviceArray(ns * cap, ecc.CORNER_DTYPE) for _ in range(2)]
    nms_cnt = [ecc.DeviceArray(ns, np.int32) for _ in range(2)]
    lib = ecc.lib
    if dist:
        # exchange buffers are torch tensors (RCCL operates on them); libecc gets their pointers
        t_counts = torch.zeros(W * H, dtype=torch.int32, device=f"cuda:{local}")
        t_local = torch.zeros(W * H, dtype=torch.int64, device=f"cuda:{local}")
        t_all = torch.zeros(world * W * H, dtype=torch.int64, device=f"cuda:{local}")

    if dist:
        t_b = torch.cuda.Stream(device=f"cuda:{local}")  # the k-means chain's stream
        ev_f, ev_j = torch.cuda.Event(), torch.cuda.Event()
        ev_cnt, ev_ar = torch.cuda.Event(), torch.cuda.Event()

    def step_sharded(nb=0, serial=args.serial):
        """Shard-local downsample/detection/NMS; global k-means from ONE all-reduce of the
        shards' per-pixel count images; exact SAE hand-off (all-gather of the shards' own last-t
        images, computed by the detection's prepare phase).  As on one GPU, the downsample ->
        k-means chain runs on a second stream beside the detection chain (--serial: one stream);
        its all-reduce is issued from that stream, before the all-gather on every rank."""
        S = ctx.stream
        main = torch.cuda.current_stream()
        if not serial:
            ev_f.record(main)
            t_b.wait_event(ev_f)
        B = S if serial else t_b.cuda_stream
        ecc.check(lib.ecc_downsample_hash(ctx.ctx, d_xy.ptr, n, ecc.C.byref(hcfg), rep_xy.ptr, None,
                                          uniq.ptr, rep.ptr, B), "downsample")
        ecc.check(lib.ecc_kmeans_counts_xy16(ctx.ctx, rep_xy.ptr, n_win, WINDOW, uniq.ptr, W, H, t_counts.data_ptr(), B))
        if native is not None:
            return step_sharded_native(nb, serial, S, B, main)
        # prepare is enqueued before the collectives: a blocking backend (gloo) waits on the host
        ecc.check(lib.ecc_fast_detect_prepare(ctx.ctx, d_xy.ptr, d_t.ptr, n, ecc.C.byref(ccfg), t_local.data_ptr(), S))
        if serial:
            dist.all_reduce(t_counts)
        else:
            with torch.cuda.stream(t_b):
                dist.all_reduce(t_counts)
        dist.all_gather_into_tensor(t_all, t_local)
        ecc.check(lib.ecc_memcpy_d2d(d_c.ptr, d_c0.ptr, 8 * K, B))
        ecc.check(lib.ecc_kmeans_run_counts(ctx.ctx, t_counts.data_ptr(), W, H, ecc.C.byref(kcfg), d_c.ptr, None, B))
        ecc.check(lib.ecc_kmeans_labels_xy16(ctx.ctx, rep_xy.ptr, n_win, WINDOW, uniq.ptr, d_c.ptr, K,
                                             kcfg.threshold, labels.ptr, B))
        if not serial:
            ev_j.record(t_b)
        ecc.check(lib.ecc_sae_max_combine(ctx.ctx, t_all.data_ptr(), rank, W * H, sae.ptr, S))
        ecc.check(lib.ecc_fast_detect_finish(ctx.ctx, d_xy.ptr, d_t.ptr, n, ecc.C.byref(ccfg), sae.ptr,
                                             flags.ptr, S), "fast_detect_finish")
        ctx.corner_nms(d_xy, flags, n, SLICE, W, H, 15, cap, nms_out[nb], nms_cnt[nb])
        if not serial:
            main.wait_event(ev_j)

    def step_sharded_native(nb, serial, S, B, main):
        """The rest of the sharded step over libecc's RCCL entry points: both collectives on the
        detection stream, in the same order on every rank (operations of one communicator must
        not overlap), the k-means chain joining through events (as apps/ecc_sharded_step.cpp)."""
        if not serial:
            ev_cnt.record(t_b)
        ecc.check(lib.ecc_fast_detect_prepare(ctx.ctx, d_xy.ptr, d_t.ptr, n, ecc.C.byref(ccfg), t_local.data_ptr(), S))
        if not serial:
            main.wait_event(ev_cnt)
        native.allreduce_counts(t_counts.data_ptr(), W * H, S)
        if not serial:
            ev_ar.record(main)
        native.sae_handoff(t_local.data_ptr(), W * H, t_all.data_ptr(), sae.ptr, S)
        if not serial:
            t_b.wait_event(ev_ar)
        ecc.check(lib.ecc_memcpy_d2d(d_c.ptr, d_c0.ptr, 8 * K, B))
        ecc.check(lib.ecc_kmeans_run_counts(ctx.ctx, t_counts.data_ptr(), W, H, ecc.C.byref(kcfg), d_c.ptr, None, B))
        ecc.check(lib.ecc_kmeans_labels_xy16(ctx.ctx, rep_xy.ptr, n_win, WINDOW, uniq.ptr, d_c.ptr, K,
                                             kcfg.threshold, labels.ptr, B))
        if not serial:
            ev_j.record(t_b)
        ecc.check(lib.ecc_fast_detect_finish(ctx.ctx, d_xy.ptr, d_t.ptr, n, ecc.C.byref(ccfg), sae.ptr,
                                             flags.ptr, S), "fast_detect_finish")
        ctx.corner_nms(d_xy, flags, n, SLICE, W, H, 15, cap, nms_out[nb], nms_cnt[nb])
        if not serial:
            main.wait_event(ev_j)

    def gather_lists(nb):
        """Shard NMS lists -> every rank: (corners, starts, counts, n_slices, keep-alive)."""
        ctx.corner_pack(nms_out[nb], nms_cnt[nb], ns, cap, packed.data_ptr(), offs.data_ptr())
        if native is not None:
            a, st_, ct_, nst = native.gather_corners(packed.data_ptr(), offs.data_ptr(), ns)
            return a.ptr, st_.ptr, ct_.ptr, nst, (a, st_, ct_)
        total_b = int(offs[-1].item())
        ecc.check(lib.ecc_memcpy_d2d(cnt_t.data_ptr(), nms_cnt[nb].ptr, 4 * ns, ctx.stream))
        pk_b, st_b, ct_b = edist.gather_corner_lists(comm, packed[:total_b], cnt_t)
        return pk_b.data_ptr(), st_b.data_ptr(), ct_b.data_ptr(), int(st_b.numel()), (pk_b, st_b, ct_b)

    # single GPU: downsample -> k-means and the corner chain read the same resident batch and are
    # independent, so they run on two streams (fork/join with events) and overlap
    s2, ev_fork, ev_join, ev_gate = ecc.P(), ecc.P(), ecc.P(), ecc.P()
    if not dist or rank == 0:  # sharded: rank 0's single-GPU rate at the same size (per_gpu_rate_n1)
        # the k-means chain's stream (a priority or a CU split for it measured no faster: DESIGN §5)
        ecc.check(lib.ecc_stream_create(ecc.C.byref(s2)), "stream")
        for e in (ev_fork, ev_join, ev_gate):
            ecc.check(lib.ecc_event_create(ecc.C.byref(e)), "event")

    def sync_all():
        """Both streams idle (a pipelined step may leave its k-means chain running)."""
        ctx.sync()
        if s2.value:
            ecc.check(lib.ecc_stream_sync(s2.value), "stream sync")

    # --corner-shards P (one GPU): the corner chain as P time-window shards of the batch on P
    # contexts and streams — the multi-GPU SAE hand-off inside one device (prepare every shard,
    # shard p starts from the max of the lower shards' own last-timestamp images, finish + NMS),
    # so the shards' kernels overlap each other's tails and low-occupancy phases
    P = max(1, args.corner_shards) if not dist else 1
    cshards = []
    if P > 1:
        HW = W * H
        cuts = [round(p * ns / P) * SLICE for p in range(P + 1)]
        c_last = ecc.DeviceArray(P * HW, np.int64)
        for p in range(P):
            cx = ctx if p == 0 else ecc.Context(local)
            cfg_p = ecc.corner_cfg(width=W, height=H, first_detect_slice=1 if p == 0 else 0)
            sae_p = sae if p == P - 1 else ecc.DeviceArray(HW, np.int64)
            evs = [ecc.P(), ecc.P()]
            for e in evs:
                ecc.check(lib.ecc_event_create(ecc.C.byref(e)), "event")
            cshards.append(dict(ctx=cx, lo=cuts[p], n=cuts[p + 1] - cuts[p], cfg=cfg_p, sae=sae_p,
                                ev_prep=evs[0], ev_done=evs[1]))

    def corner_chain_shards(nb):
        main = ctx.stream
        for p, c in enumerate(cshards):
            S = c["ctx"].stream
            if p > 0:
                ecc.check(lib.ecc_stream_wait_event(S, ev_fork))
            ecc.check(lib.ecc_fast_detect_prepare(c["ctx"].ctx, d_xy.ptr + 4 * c["lo"], d_t.ptr + 8 * c["lo"], c["n"],
                                                  ecc.C.byref(c["cfg"]), c_last.ptr + 8 * p * W * H, S), "prepare")
            ecc.check(lib.ecc_event_record(c["ev_prep"], S))
        for p, c in enumerate(cshards):
            S, cx = c["ctx"].stream, c["ctx"].ctx
            for q in range(p):
                ecc.check(lib.ecc_stream_wait_event(S, cshards[q]["ev_prep"]))
            # the SAE at the shard's start: the step's initial SAE is zero (memset), so the max
            # of the lower shards' own last images
            ecc.check(lib.ecc_sae_max_combine(cx, c_last.ptr, p, W * H, c["sae"].ptr, S), "sae combine")
            s0 = c["lo"] // SLICE
            ecc.check(lib.ecc_fast_detect_finish_nms(cx, d_xy.ptr + 4 * c["lo"], d_t.ptr + 8 * c["lo"], c["n"],
                                                     ecc.C.byref(c["cfg"]), c["sae"].ptr, flags.ptr + c["lo"], 15,
                                                     cap, nms_out[nb].ptr + s0 * cap * ecc.CORNER_DTYPE.itemsize,
                                                     nms_cnt[nb].ptr + 4 * s0, S), "finish_nms")
            if p > 0:
                ecc.check(lib.ecc_event_record(c["ev_done"], S))
                ecc.check(lib.ecc_stream_wait_event(main, c["ev_done"]))

    def step(serial=args.serial, nb=0):
        if dist:
            # gloo collectives block the host, so its timing runs keep one stream (measured faster);
            # --overlap keeps the two-stream schedule for correctness rehearsals
            return step_sharded(nb, serial or (args.dist_backend != "nccl" and not args.overlap))
        return step_single(serial, nb)

    pipelined = not (args.joined or args.graph or P > 1)

    def step_single(serial=args.serial, nb=0):
        """The single-GPU step: downsample -> k-means on the second stream beside detect + NMS.
        Pipelined (default): the detection is split at its sort phase (prepare | finish + NMS),
        the k-means passes wait for that point, and the step does not wait for the k-means
        stream, so step i's k-means chain overlaps step i+1's detection (a stream of batches as a
        host would feed it); every step still runs every stage on its own batch, and the timed
        region ends only when both streams are idle.  --joined: the per-step fork/join."""
        ks = ctx.stream if serial else s2.value  # the k-means chain's stream
        ecc.check(lib.ecc_event_record(ev_fork, ctx.stream))
        ecc.check(lib.ecc_stream_wait_event(ks, ev_fork))
        if pipelined and not serial:
            ecc.check(lib.ecc_downsample_hash(ctx.ctx, d_xy.ptr, n, ecc.C.byref(hcfg), rep_xy.ptr, None,
                                              uniq.ptr, rep.ptr, ks), "downsample")
            ecc.check(lib.ecc_memset_async(sae.ptr, 0, sae.nbytes, ctx.stream))
            ecc.check(lib.ecc_fast_detect_prepare(ctx.ctx, d_xy.ptr, d_t.ptr, n, ecc.C.byref(ccfg), None, ctx.stream),
                      "fast_detect_prepare")
            ecc.check(lib.ecc_event_record(ev_gate, ctx.stream))  # the sort phase is enqueued
            ecc.check(lib.ecc_stream_wait_event(ks, ev_gate))
            ecc.check(lib.ecc_memcpy_d2d(d_c.ptr, d_c0.ptr, 8 * K, ks))
            ecc.check(lib.ecc_kmeans_run_xy16_frame(ctx.ctx, rep_xy.ptr, n_win, WINDOW, uniq.ptr, W, H,
                                                    ecc.C.byref(kcfg), d_c.ptr, labels.ptr, None, ks), "kmeans")
            ecc.check(lib.ecc_fast_detect_finish_nms(ctx.ctx, d_xy.ptr, d_t.ptr, n, ecc.C.byref(ccfg), sae.ptr,
                                                     flags.ptr, 15, cap, nms_out[nb].ptr, nms_cnt[nb].ptr,
                                                     ctx.stream), "fast_detect_finish_nms")
            return
        ecc.check(lib.ecc_downsample_hash(ctx.ctx, d_xy.ptr, n, ecc.C.byref(hcfg), rep_xy.ptr, None,
                                          uniq.ptr, rep.ptr, ks), "downsample")
        ecc.check(lib.ecc_memcpy_d2d(d_c.ptr, d_c0.ptr, 8 * K, ks))
        ecc.check(lib.ecc_kmeans_run_xy16_frame(ctx.ctx, rep_xy.ptr, n_win, WINDOW, uniq.ptr, W, H, ecc.C.byref(kcfg),
                                                d_c.ptr, labels.ptr, None, ks), "kmeans")
        ecc.check(lib.ecc_event_record(ev_join, ks))
        if cshards and not serial:
            corner_chain_shards(nb)  # every shard's SAE is derived from zero (the memset below)
        else:
            ecc.check(lib.ecc_memset_async(sae.ptr, 0, sae.nbytes, ctx.stream))
            # detect + per-slice NMS in one call: the flag pass writes the NMS candidate lists
            ctx.fast_detect_nms(d_xy, d_t, n, ccfg, sae, flags, 15, cap, nms_out[nb], nms_cnt[nb])
        ecc.check(lib.ecc_stream_wait_event(ctx.stream, ev_join))

    for _ in range(args.warmup):
        step()
    sync_all()
    for cx in [ctx] + [c["ctx"] for c in cshards[1:]]:
        cx.sync()
        if cx.fast_detect_status() != 0:
            raise RuntimeError("fast_detect reported a status error")
        if cx.corner_nms_status() != 0:
            raise RuntimeError("corner_nms reported a status error")
    if dist and lib.ecc_kmeans_counts_status(ctx.ctx, ctx.stream) != 0:
        raise RuntimeError("a representative lies outside the k-means count frame")

    # sharded runs: rank 0's single-GPU rate at the same per-GPU size, measured in this job before
    # the sharded timed region (the other ranks wait at the barrier), so that the line itself
    # carries the N=1 reference of its scaling efficiency
    per_gpu_rate_n1 = None
    if dist and rank == 0 and not args.no_n1_rate:
        for _ in range(max(1, args.warmup)):
            step_single(args.serial)
        sync_all()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_single(args.serial)
        sync_all()
        dt1 = time.perf_counter() - t0
        if ctx.fast_detect_status() != 0 or ctx.corner_nms_status() != 0:
            raise RuntimeError("single-GPU reference steps reported a status error")
        per_gpu_rate_n1 = {"value": round(args.steps * n / dt1 / 1e6, 2), "unit": "Mevents/s",
                           "ms_per_step": round(dt1 / args.steps * 1e3, 3), "events_per_gpu": n,
                           "how": "rank 0, the single-GPU two-stream step (no collectives) over the same "
                                  f"{n}-event shard, {args.steps} steps after warm-up, in this job"}
    if dist:
        dist.barrier()
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
        sync_all()

    def timed_step():
        if graph is not None:
            ecc.check(lib.ecc_graph_launch(graph, ctx.stream), "ecc_graph_launch")
        else:
            step()

    # 1. the timed region: K steps, uninstrumented (a timestamped HIP event around every launch
    #    drains the queue between kernels and costs ~0.6 ms/step here)
    if dist:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        timed_step()
    sync_all()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_step = elapsed / args.steps * 1e3

    # 2. the kernel-timing pass: the same K steps again with HIP events recorded around every
    #    launch on its stream (ecc_ctx_set_timing) -> per-kernel average durations.  It runs on
    #    ONE stream, so that a kernel's time is its own (not queueing behind the other chain).
    lib.ecc_ctx_set_timing(ctx.ctx, 1)
    lib.ecc_ctx_timing_reset(ctx.ctx)
    sync_all()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step(serial=True)
    sync_all()
    instrumented = time.perf_counter() - t1
    lib.ecc_ctx_set_timing(ctx.ctx, 0)
    stats = ctx.timing_report()
    detect_stats = ctx.fast_detect_stats()

    # ---- roofline (SURVEY.md §8d algorithmic bytes per unit) ------------------------------------
    kern_ms = {k: v["total_ms"] for k, v in stats.items()}
    dominant = max(kern_ms, key=kern_ms.get)
    launches = stats[dominant]["launches"]
    avg_ms = kern_ms[dominant] / launches

    def stage_ms(names):
        return sum(kern_ms.get(k, 0.0) for k in names) / args.steps

    # §8d: downsample 4 B/event in + 4 B/rep out + 8 B/window; k-means 8 B/point/iteration
    # (float2 read) + 1 B/point (final label); SAE + arc test 12 B/event in (xy + t) + 1 B/event
    # out (corner flag); NMS and tracker are latency work (reported in µs, no roofline).
    bytes_stage = {
        "downsample": 4.0 * n + 4.0 * n_reps + 8.0 * n_win,
        "kmeans": (8.0 * I + 1.0) * n_reps,
        "corner": 13.0 * n,
    }
    t_stage = {
        "downsample": stage_ms(("downsample_hash_kernel",)),
        "kmeans": stage_ms(KMEANS_KERNELS),
        "corner": stage_ms(CORNER_KERNELS),
    }
    stages = {}
    for k in bytes_stage:
        ach = bytes_stage[k] / (t_stage[k] * 1e-3) / 1e9 if t_stage[k] > 0 else 0.0
        stages[k] = {"ms_per_step": round(t_stage[k], 4), "algorithmic_bytes": bytes_stage[k],
                     "achieved_gbs": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4)}
    # the count-image k-means reads a representative twice (count, labels: 4 + 4 B) and writes its
    # label (1 B); its Lloyd passes run over the 90 K-pixel image and never move §8d's per-pass
    # point bytes.  Its roofline is therefore on those 9 B/point; §8d's figure stays only as a
    # normalised rate (point-passes per second), which is NOT a roofline
    if t_stage["kmeans"] > 0:
        own = 9.0 * n_reps
        ach = own / (t_stage["kmeans"] * 1e-3) / 1e9
        stages["kmeans"] = {
            "ms_per_step": round(t_stage["kmeans"], 4), "algorithmic_bytes": own, "achieved_gbs": round(ach, 1),
            "frac": round(ach / HBM_PEAK_GBS, 4), "bound": "latency (ten dependent Lloyd launches)",
            "bytes_note": "9 B/representative: 4 B read by the count pass, 4 B by the label pass, 1 B label",
            "gpoint_passes_s": round(n_reps * (I + 1) / (t_stage["kmeans"] * 1e-3) / 1e9, 2)}
    e2e_bytes = sum(bytes_stage.values())
    # the bytes this pipeline must actually move: the count-image k-means never moves §8d's
    # 8 B/point/pass, so its 9 B/representative replace them (downsample + k-means + corner)
    pipe_bytes = bytes_stage["downsample"] + 9.0 * n_reps + bytes_stage["corner"]
    stages["nms"] = {"ms_per_step": round(stage_ms(NMS_KERNELS), 4), "bound": "latency"}
    pipe_gbs = pipe_bytes / (ms_step * 1e-3) / 1e9
    s8d_gbs = e2e_bytes / (ms_step * 1e-3) / 1e9
    stages["e2e"] = {"ms_per_step": round(ms_step, 4),
                     "pipeline_bytes": pipe_bytes, "achieved_gbs": round(pipe_gbs, 1),
                     "frac": round(pipe_gbs / HBM_PEAK_GBS, 4),
                     "algorithmic_bytes_s8d": e2e_bytes, "achieved_gbs_s8d": round(s8d_gbs, 1),
                     "frac_s8d": round(s8d_gbs / HBM_PEAK_GBS, 4),
                     "note": "wall time of the whole step (both streams).  frac: over the bytes the pipeline "
                             "moves (downsample 4 B/event + 4 B/rep + 8 B/window, k-means 9 B/rep, corner "
                             "13 B/event); frac_s8d: over SURVEY §8d's stage bytes, whose k-means term "
                             "(8 B/point/pass x 10 passes) the count-image form never moves"}
    # the dominant kernel carries its stage's §8d bytes (the corner stage's 13 B/event for the arc
    # kernel): what that stage must move at minimum, over this one kernel's launch time
    stage_of = {**{k: "corner" for k in CORNER_KERNELS}, **{k: "kmeans" for k in KMEANS_KERNELS},
                "downsample_hash_kernel": "downsample"}
    dom_stage = stage_of.get(dominant)
    bytes_per_launch = bytes_stage[dom_stage] if dom_stage else 0.0
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    # HBM bytes per launch of the same kernel from the newest committed PMC summary
    # (scripts/gpu_evidence.sh + scripts/traffic.py; PMC passes cannot run inside this process)
    traffic = None
    traffic_src = None
    tfiles = sorted((ROOT / "profiles").glob("*_traffic.json"))
    if tfiles:
        try:
            rec = json.loads(tfiles[-1].read_text()).get(dominant)
            traffic = round(rec["bytes_per_launch"]) if rec else None
            traffic_src = tfiles[-1].name
        except (ValueError, KeyError, TypeError):
            traffic = None
    # the line's frac is this run's own HIP-event figure.  Beside it: the same kernel's average
    # from a committed rocprofv3 --stats summary, only when that trace was taken with THIS
    # library (its meta file records the libecc sha256; scripts/gpu_evidence.sh writes it)
    rp_ms, rp_src = rocprof_avg_ms(dominant, lib_sha256(ecc))

    # ---- tracker (sequential over slices, rank 0 of a 1-GPU run) ---------------------------------
    tracker = None
    g_tracker = None
    if not args.no_tracker and not dist:
        tr = ecc.Tracker(ctx)
        tmr = ecc.Timer(ctx.stream)
        tmr.start()
        tr.update(nms_out[0], nms_cnt[0], ns, cap)
        trk_ms = tmr.stop()
        if tr.status() != 0:
            raise RuntimeError("tracker reported a status error")
        g_tracker = (tr.tracks(), tr.groups()[0])
        tr.close()
        # pipelined: the tracker of batch b (stream 3) overlaps the detection of batch b+1; the
        # NMS buffers alternate, and batch b+2 waits for the tracker of batch b to release one
        s3 = ecc.P()
        ecc.check(lib.ecc_stream_create(ecc.C.byref(s3)), "stream")
        ev_nms = [ecc.P(), ecc.P()]
        ev_trk = [ecc.P(), ecc.P()]
        for e in ev_nms + ev_trk:
            ecc.check(lib.ecc_event_create(ecc.C.byref(e)), "event")
        trp = ecc.Tracker(ctx)
        kp = max(3, min(args.steps, 6))
        sync_all()
        tp0 = time.perf_counter()
        for b in range(kp):
            nb = b % 2
            if b >= 2:
                ecc.check(lib.ecc_stream_wait_event(ctx.stream, ev_trk[nb]))
            step(nb=nb)
            ecc.check(lib.ecc_event_record(ev_nms[nb], ctx.stream))
            ecc.check(lib.ecc_stream_wait_event(s3.value, ev_nms[nb]))
            ecc.check(lib.ecc_tracker_update(trp.tr, nms_out[nb].ptr, nms_cnt[nb].ptr, ns, cap, s3.value))
            ecc.check(lib.ecc_event_record(ev_trk[nb], s3.value))
        ecc.check(lib.ecc_stream_sync(s3.value))
        sync_all()
        tp = time.perf_counter() - tp0
        trp.close()
        tracker = {
            "slices": ns, "us_per_slice": round(trk_ms * 1e3 / ns, 2), "ms_per_batch": round(trk_ms, 3),
            "tracks_end": len(g_tracker[0]), "groups_end": len(g_tracker[1]),
            "with_tracker": {"mevents_s": round(kp * n / tp / 1e6, 1), "ms_per_step": round(tp / kp * 1e3, 3),
                             "steps": kp,
                             "how": "tracker of batch b on a third stream overlapping detection of batch b+1"},
        }

    # ---- C5 track merge: shard NMS lists gathered in global slice order -> ONE tracker (rank 0) ----
    track_merge = None
    merged_tracks = None
    if dist and not args.no_tracker:
        from eccpy import dist as edist
        comm = edist.TorchComm(dist)
        packed = torch.zeros((ns * cap, 3), dtype=torch.int32, device=f"cuda:{local}")
        offs = torch.zeros(ns + 1, dtype=torch.int64, device=f"cuda:{local}")
        cnt_t = torch.empty(ns, dtype=torch.int32, device=f"cuda:{local}")
        dist.barrier()
        sync_all()
        tm0 = time.perf_counter()
        pk_p, st_p, ct_p, n_gs, keep = gather_lists(0)
        sync_all()
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tm0) * 1e3
        if rank == 0:
            tr = ecc.Tracker(ctx)
            tmr = ecc.Timer(ctx.stream)
            tmr.start()
            tr.update_lists(pk_p, st_p, ct_p, n_gs)
            merge_ms = tmr.stop()
            if tr.status() != 0:
                raise RuntimeError("merged tracker reported a status error")
            cts = keep[2].numpy() if native is not None else keep[2].cpu().numpy()
            n_corners = int(cts[:n_gs].astype(np.int64).sum())
            track_merge = {"ranks": world, "slices": n_gs, "corners": n_corners,
                           "transport": "ecc_dist_* (libecc RCCL)" if native is not None else "torch.distributed",
                           "pack_gather_ms": round(gather_ms, 3), "tracker_ms": round(merge_ms, 3),
                           "us_per_slice": round(merge_ms * 1e3 / n_gs, 2),
                           "tracks_end": len(tr.tracks())}
            merged_tracks = (tr.tracks(), tr.groups()[0])
            tr.close()
        dist.barrier()
        # pipelined: the merged tracker of step b (rank 0, third stream) overlaps the sharded step
        # b+1 on every rank; per step the shards' lists are packed and gathered (host-synchronising:
        # the gather needs the list sizes).  Whole-job events / wall time of the loop.
        s3, ev_g, ev_trk = ecc.P(), [ecc.P(), ecc.P()], [ecc.P(), ecc.P()]
        ecc.check(lib.ecc_stream_create(ecc.C.byref(s3)), "stream")
        for e in ev_g + ev_trk:
            ecc.check(lib.ecc_event_create(ecc.C.byref(e)), "event")
        trp = ecc.Tracker(ctx) if rank == 0 else None
        held = [None, None]
        kp = max(3, min(args.steps, 6))
        dist.barrier()
        sync_all()
        tp0 = time.perf_counter()
        for b in range(kp):
            nb = b % 2
            if b >= 2 and rank == 0:  # the gathered lists of step b-2 are released after their tracker
                ecc.check(lib.ecc_stream_wait_event(ctx.stream, ev_trk[nb]))
            step(nb=nb)
            held[nb] = gather_lists(nb)
            if rank == 0:
                pk_p, st_p, ct_p, n_gs, _ = held[nb]
                ecc.check(lib.ecc_event_record(ev_g[nb], ctx.stream))
                ecc.check(lib.ecc_stream_wait_event(s3.value, ev_g[nb]))
                ecc.check(lib.ecc_tracker_update_lists(trp.tr, pk_p, st_p, ct_p, n_gs, s3.value), "tracker lists")
                ecc.check(lib.ecc_event_record(ev_trk[nb], s3.value))
        ecc.check(lib.ecc_stream_sync(s3.value))
        sync_all()
        dist.barrier()
        tp = time.perf_counter() - tp0
        if rank == 0:
            if trp.status() != 0:
                raise RuntimeError("pipelined merged tracker reported a status error")
            track_merge["pipelined"] = {
                "mevents_s": round(world * kp * n / tp / 1e6, 1), "ms_per_step": round(tp / kp * 1e3, 3),
                "steps": kp, "how": "sharded step b+1 on every rank while rank 0's tracker consumes the gathered "
                                    "lists of step b on a third stream; pack + gather per step"}
            trp.close()
        held = [None, None]
    dist_parity = None
    if dist and args.dist_parity:
        dist_parity = shard_parity(ecc, args, dist, torch, rank, world, local, W, H, I, c0,
                                   dict(flags=flags, sae=sae, c=d_c, nms_out=nms_out[0], nms_cnt=nms_cnt[0], cap=cap,
                                        tracker=merged_tracks))

    # ---- RAW ingest, reported beside the headline ------------------------
    ingest = None
    if not args.no_ingest and rank == 0:
        ingest = bench_ingest(ecc, ctx, args, xy_h, t_h, p_h, n)

    # ---- eps-neighbourhoods + DBSCAN (BASELINE C4) --------------------
    eps_res = None
    if not args.no_eps and rank == 0:
        eps_res = bench_eps(ecc, ctx, args, rep_xy, uniq, n_win, n_reps)
        eps_res["optics_published_workloads"] = bench_optics_published(ecc, ctx)

    # ---- BASELINE C3: k-means k=16 on 50 M points (the step's representatives tiled) -------------
    c3_res = None
    if not args.no_c3 and rank == 0:
        c3_res = bench_c3(ecc, ctx, args, rep_xy, uniq, c0, K)

    value = world * args.steps * n / elapsed / 1e6
    preset = next((k for k, v in PRESET_SLICES.items() if v * SLICE == n), None)
    cname = {"c4": "BASELINE configs C2-C4", "c5": "BASELINE C5 per-GPU share"}.get(preset, "custom size")
    if world > 1:
        wl = (f"C5: {world}xMI355X time-window shards of a {world * n}-event stream ({n} events/GPU; "
              f"{cname}); per shard: ")
    else:
        wl = ""
    if graph is not None:
        lib.ecc_graph_destroy(graph)
    result = {
        "metric": "Mevents/s (downsample+cluster+corner)",
        "value": round(value, 2),
        "unit": "Mevents/s",
        "n_gpus": world,
        "dist_world": dist.get_world_size() if dist else None,
        "dist_backend": ("ecc_dist (libecc RCCL) + gloo control plane" if native is not None else args.dist_backend)
                        if dist else None,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16xy/i64t (int), fp32 k-means",
        "data": "synthetic (seeded splitmix64 event generator: moving polygons + Gaussian blobs + noise)",
        "config": {
            "workload": wl + f"e2e hash-downsample(8192-event windows) -> k-means k={K} ({I} iters) on reps -> "
                             f"SAE+FAST arc corners (16384-event slices) -> 15x15 NMS; {W}x{H} sensor; "
                             f"{n} events/GPU/step ({cname})",
            "events_per_gpu": n, "events_total": world * n, "preset": preset,
            "reps_per_gpu": n_reps, "width": W, "height": H, "k": K,
            "kmeans_iters": I, "parallelism": f"time-window shards x{world}",
            "launch": "hipGraph replay of the captured step" if graph is not None else "eager launches",
            "streams": "two streams sharing all CUs" if not (dist or args.serial) else "see parallelism",
            "schedule": ("pipelined: the k-means passes of step i start after its sort phase and may overlap step "
                         "i+1's detection; the timed region ends when both streams are idle")
                        if (pipelined and not dist and not args.serial) else "joined (per-step fork/join)",
            "corner_shards": P,
        },
        "roofline": {
            "kernel": dominant, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "avg_launch_ms": round(avg_ms, 5), "frac_from": "HIP events (this run)",
            "rocprof_avg_launch_ms": round(rp_ms, 5) if rp_ms else None, "rocprof_source": rp_src,
            "frac_rocprof": round(bytes_per_launch / (rp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if rp_ms else None,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "algorithmic_bytes": f"SURVEY §8d bytes of the kernel's stage ({dom_stage})",
            "traffic_source": traffic_src,
            "timing": f"HIP events around every launch in a second, eager, one-stream {args.steps}-step "
                      f"pass ({instrumented / args.steps * 1e3:.3f} ms/step instrumented)",
        },
        "stages": stages,
        "stages_ms_per_step": {k: round(v / args.steps, 4) for k, v in sorted(kern_ms.items())},
        "corner_items": detect_stats,
        "tracker": tracker,
        "track_merge": track_merge,
        "per_gpu_rate_n1": per_gpu_rate_n1,
        "dist_parity": dist_parity,
        "ingest": ingest,
        "eps": eps_res,
        "kmeans_c3": c3_res,
    }
    if rank == 0 and not dist and not args.no_cpu:
        base, par = cpu_leg(ecc, args, W, H, K, I, xy_h, t_h, n, c0, ctx,
                            dict(rep_xy=rep_xy, uniq=uniq, rep=rep, c=d_c, labels=labels, flags=flags, sae=sae,
                                 nms_out=nms_out[0], nms_cnt=nms_cnt[0], cap=cap, tracker=g_tracker))
        result["cpu_baseline"] = base
        result["parity"] = par
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        if native is not None:
            native.close()
        dist.destroy_process_group()


def lib_sha256(ecc):
    import hashlib
    try:
        return hashlib.sha256(Path(ecc.LIB_PATH).read_bytes()).hexdigest()
    except OSError:
        return None


def rocprof_avg_ms(kernel, sha):
    """(average ms per launch, file) of `kernel` (libecc's timing name) in the newest
    profiles/*_kernel_stats.csv that lists it AND whose meta file
    (<same stem>.meta.json, {"libecc_sha256": ...}) names the loaded library, or (None, None)."""
    import csv
    import re
    for f in sorted((ROOT / "profiles").glob("r*_kernel_stats.csv"), reverse=True):
        if "kmeans_f32" in f.name:
            continue
        try:
            meta = json.loads(f.with_name(f.name[:-len(".csv")] + ".meta.json").read_text())
        except (OSError, ValueError):
            continue
        if not sha or meta.get("libecc_sha256") != sha:
            continue
        try:
            for r in csv.DictReader(open(f)):
                m = re.search(r"::([A-Za-z_0-9]+)(<[^>]*>)?\(", r["Name"])
                if m and m.group(1) == kernel:
                    return float(r["AverageNs"]) * 1e-6, f.name
        except (OSError, KeyError, ValueError):
            continue
    return None, None


def timed_kernels(ctx, run, reps):
    """(ms per call over `reps` uninstrumented calls, per-kernel average ms from an instrumented
    pass of the same calls)."""
    import eccpy as ecc
    run()
    ctx.sync()
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
    return call_ms, {k: v["total_ms"] / v["launches"] for k, v in st.items()}


def bench_ingest(ecc, ctx, args, xy_h, t_h, p_h, n):
    """The same events written as EVT 3.0 / EVT 2.0 words, decoded from device-resident words."""
    ingest = {}
    for fmt, name in ((ecc.EVT3, "EVT3"), (ecc.EVT2, "EVT2")):
        words = ecc.evt_encode(fmt, xy_h, t_h, p_h)
        d_words = ecc.DeviceArray.from_numpy(words, ctx.stream)
        d_oxy, d_ot = ecc.DeviceArray(n, np.uint32), ecc.DeviceArray(n, np.int64)
        d_op, d_on = ecc.DeviceArray(n, np.uint8), ecc.DeviceArray(1, np.int64)
        dec_ms, kern = timed_kernels(ctx, lambda: ctx.evt_decode(fmt, d_words, len(words), d_oxy, d_ot, d_op, n, d_on),
                                     max(args.steps, 5))
        assert int(d_on.numpy()[0]) == n and ctx.evt_status() == 0
        dk = kern.get("evt_decode_kernel", float("nan"))
        ach = (words.nbytes + 13.0 * n) / (dk * 1e-3) / 1e9  # words in + xy/t/p out
        ingest[name] = {
            "words": len(words), "word_bytes": words.itemsize, "events": n,
            "mevents_s": round(n / (dec_ms * 1e-3) / 1e6, 1), "ms_per_decode": round(dec_ms, 4),
            "kernels_us": {k: round(v * 1e3, 2) for k, v in sorted(kern.items())},
            "roofline": {"kernel": "evt_decode_kernel", "bound": "hbm", "achieved": round(ach, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes": f"{words.itemsize} B/word in + 13 B/event out"},
        }
        del d_words, d_oxy, d_ot, d_op, d_on
    return ingest


def bench_c3(ecc, ctx, args, rep_xy, uniq, c0, K, n_pts=50_000_000):
    """BASELINE C3: k-means k=16 on 50 M points (this step's C2-style representatives tiled to
    50 M), 10 Lloyd passes + final labels, three ways: packed-u16 points through the per-pixel
    count path, and float points through the vector and the two matrix-core assignment engines
    (4x4x1 per-lane form, 32x32x2 streaming form).
    Roofline per SURVEY §8d: 8 B/point/iteration (float2 read) + 1 B/point (labels)."""
    u = uniq.numpy()
    rx = rep_xy.numpy()
    dense = np.concatenate([rx[w * WINDOW: w * WINDOW + u[w]] for w in range(len(u))])
    pts = np.resize(dense, n_pts)
    x, y = ecc.unpack_xy(pts)
    f = np.empty(2 * n_pts, np.float32)
    f[0::2], f[1::2] = x, y
    d_pts, d_f = ecc.DeviceArray.from_numpy(pts, ctx.stream), ecc.DeviceArray.from_numpy(f, ctx.stream)
    del f
    d_c0 = ecc.DeviceArray.from_numpy(c0, ctx.stream)
    d_c = ecc.DeviceArray(2 * K, np.float32)
    d_lab = ecc.DeviceArray(n_pts, np.uint8)
    I = 10
    cfg = ecc.kmeans_cfg(k=K, max_iters=I, tol=-1.0)
    lib = ecc.lib
    alg = (8.0 * I + 1.0) * n_pts
    out = {"points": n_pts, "k": K, "iters": I, "algorithmic_bytes": alg,
           "algorithmic": "8 B/point/iteration (float2) + 1 B/point labels (SURVEY 8d)"}
    results = {}
    for name, run in (
            ("xy16_count_image", lambda: ctx.kmeans_xy16_frame(d_pts, 1, n_pts, None, 346, 260, d_c, cfg, d_lab)),
            ("f32_vector", lambda: ctx.kmeans_f32_engine(d_f, n_pts, d_c, cfg, 1, d_lab)),
            ("f32_mfma", lambda: ctx.kmeans_f32_engine(d_f, n_pts, d_c, cfg, 2, d_lab)),
            ("f32_mfma_32x32x2", lambda: ctx.kmeans_f32_engine(d_f, n_pts, d_c, cfg, 3, d_lab))):
        def full():
            ecc.check(lib.ecc_memcpy_d2d(d_c.ptr, d_c0.ptr, 8 * K, ctx.stream))
            run()
        ms, kern = timed_kernels(ctx, full, 3)
        cen = d_c.numpy().copy()
        # the count-image form reads each point twice (count, labels: 4 + 4 B) and writes its
        # label (1 B); its passes run over the 90 K-pixel image, so §8d's per-iteration point
        # bytes would put it above the HBM peak — its frac is on the bytes it must move
        own = 9.0 * n_pts if name == "xy16_count_image" else alg
        ach = own / (ms * 1e-3) / 1e9
        results[name] = cen
        out[name] = {"ms": round(ms, 3), "mpoints_s": round(n_pts / (ms * 1e-3) / 1e6, 1),
                     "algorithmic_bytes": own, "achieved_gbs": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                     "gpoint_passes_s": round(n_pts * (I + 1) / (ms * 1e-3) / 1e9, 2),
                     "kernels_us": {k: round(v * 1e3, 2) for k, v in sorted(kern.items())}}
    # the three forms agree bit for bit (integer-valued points: exact fp64 / integer sums)
    out["centroids_agree"] = bool(all(np.array_equal(results[a].view(np.uint32), results["f32_vector"].view(np.uint32))
                                      for a in results))
    f32 = {k: out[k]["ms"] for k in ("f32_vector", "f32_mfma", "f32_mfma_32x32x2")}
    out["winner_f32"] = min(f32, key=f32.get)
    out["winner"] = min(("xy16_count_image", *f32), key=lambda k: out[k]["ms"])
    return out


def bench_eps(ecc, ctx, args, rep_xy, uniq, n_win, n_reps):
    """Per 8192-event downsample window over the step's device-resident representatives:
    DBSCAN eps 20 / minPts 20 (PCC/pcl_cluster.cpp:113-120) — counts, lists, cluster
    extraction — and OPTICS eps 10 / min_pts 2 (OPT/test/cluster_event_data.cpp:449) — counts
    + core distances."""
    res = {}
    reps = max(args.steps, 5)
    tot = n_win * WINDOW
    e_cnt = ecc.DeviceArray(tot, np.int32)
    e_core = ecc.DeviceArray(tot, np.float64)
    for name, eps, mp, core in (("dbscan_eps20_minpts20", 20.0, 20, None),
                                ("optics_eps10_minpts2", 10.0, 2, e_core)):
        call_ms, kern = timed_kernels(ctx, lambda: ctx.eps_counts(rep_xy, n_win, WINDOW, uniq, eps, mp, e_cnt, core), reps)
        # the counts are eps_run_counts_kernel (+ the candidate walk over its leftover segments), or
        # eps_counts_kernel alone with core distances
        ck = [k for k in ("eps_run_counts_kernel", "eps_counts_left_kernel", "eps_counts_kernel") if k in kern]
        ek = sum(kern[k] for k in ck) if ck else float("nan")
        per_rep = 8 + (8 if core is not None else 0)  # xy in + count out [+ core distance out]
        ach = n_reps * per_rep / (ek * 1e-3) / 1e9
        res[name] = {
            "reps": n_reps, "windows": n_win, "mreps_s": round(n_reps / (call_ms * 1e-3) / 1e6, 1),
            "ms_per_call": round(call_ms, 4), "kernels_us": {k: round(v * 1e3, 2) for k, v in sorted(kern.items())},
            "roofline": {"kernel": "+".join(ck), "bound": "hbm", "achieved": round(ach, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes": f"4 B/rep in + 4 B/rep out{' + 8 B/rep core distance' if core is not None else ''}"},
        }
    # the full DBSCAN chain (eps 20 / minPts 20, clusters of 100..25000): counts -> ascending
    # neighbour lists -> union-find extraction (DBSCAN_simple.h:27-90)
    ctx.eps_counts(rep_xy, n_win, WINDOW, uniq, 20.0, 20, e_cnt, None)
    d_off = ecc.DeviceArray(tot + 1, np.int64)
    ctx.sync()
    cnt = e_cnt.numpy()
    u = uniq.numpy()
    valid = (np.arange(WINDOW)[None, :] < u[:, None]).ravel()
    nbr_cap = int(cnt[valid].sum()) + 16
    d_nbr = ecc.DeviceArray(nbr_cap, np.int32)
    d_lab = ecc.DeviceArray(tot, np.int32)
    d_nc = ecc.DeviceArray(n_win, np.int32)
    dup_cap = 1 << 22
    d_dups = ecc.DeviceArray(2 * dup_cap, np.int64)
    d_nd = ecc.DeviceArray(1, np.int64)

    def chain():
        ctx.eps_counts(rep_xy, n_win, WINDOW, uniq, 20.0, 20, e_cnt, None)
        ctx.eps_lists(rep_xy, n_win, WINDOW, uniq, 20.0, e_cnt, d_off, d_nbr, nbr_cap)
        ctx.dbscan_extract(n_win, WINDOW, uniq, d_off, d_nbr, 20, 100, 25000, d_lab, d_nc, d_dups, dup_cap, d_nd)

    chain_ms, kern = timed_kernels(ctx, chain, max(3, min(reps, 5)))
    st = ctx.dbscan_status()
    nc = d_nc.numpy()
    res["dbscan_chain_eps20_minpts20"] = {
        "reps": n_reps, "windows": n_win, "ms_per_call": round(chain_ms, 4),
        "us_per_window": round(chain_ms * 1e3 / n_win, 3), "mreps_s": round(n_reps / (chain_ms * 1e-3) / 1e6, 1),
        "neighbour_entries": nbr_cap - 16, "clusters": int(nc.sum()), "status": st,
        "kernels_us": {k: round(v * 1e3, 2) for k, v in sorted(kern.items())},
    }
    # the same DBSCAN fused (ecc_dbscan_grid: no lists, one launch); its clusters must equal the
    # chain's (labels, cluster counts, duplicate memberships as a set)
    lab_chain, nd_chain = d_lab.numpy().copy(), int(d_nd.numpy()[0])
    dups_chain = d_dups.numpy()[:2 * min(nd_chain, dup_cap)].reshape(-1, 2)
    g_lab = ecc.DeviceArray(tot, np.int32)
    g_nc = ecc.DeviceArray(n_win, np.int32)
    g_nd = ecc.DeviceArray(1, np.int64)
    grid_ms, kern = timed_kernels(ctx, lambda: ctx.dbscan_grid(rep_xy, n_win, WINDOW, uniq, 20.0, 20, 100, 25000,
                                                               g_lab, g_nc, d_dups, dup_cap, g_nd), reps)
    st_g = ctx.dbscan_status()
    nd_g = int(g_nd.numpy()[0])
    dups_g = d_dups.numpy()[:2 * min(nd_g, dup_cap)].reshape(-1, 2)
    same = (np.array_equal(g_lab.numpy()[valid], lab_chain[valid]) and np.array_equal(g_nc.numpy(), nc)
            and nd_g == nd_chain and set(map(tuple, dups_g.tolist())) == set(map(tuple, dups_chain.tolist())))
    # the row-run kernel (distinct-pixel windows) + the cell-grid kernel over what it leaves
    gks = [k for k in ("dbscan_run_kernel", "dbscan_grid_left_kernel", "dbscan_grid_kernel") if k in kern]
    gk = sum(kern[k] for k in gks) if gks else float("nan")
    res["dbscan_grid_eps20_minpts20"] = {
        "reps": n_reps, "windows": n_win, "ms_per_call": round(grid_ms, 4),
        "us_per_window": round(grid_ms * 1e3 / n_win, 3), "mreps_s": round(n_reps / (grid_ms * 1e-3) / 1e6, 1),
        "clusters": int(g_nc.numpy().sum()), "dup_memberships": nd_g, "status": st_g,
        "equals_chain": bool(same),
        "kernels_us": {k: round(v * 1e3, 2) for k, v in sorted(kern.items())},
        "roofline": {"kernel": "+".join(gks), "bound": "hbm",
                     "achieved": round(n_reps * 8 / (gk * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(n_reps * 8 / (gk * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "algorithmic_bytes": "4 B/rep in + 4 B/rep label out"},
    }
    return res


# The only published timings of the reference: the vendored OPTICS library's benchmark
# (OPT/test/Benchmark/benchmark.cpp:62-226 -> Benchmark.ods): uniform random
# doubles in the unit hypercube, compute_reachability_dists with auto-epsilon, mean of 2 laps,
# on an Intel Xeon E3-1225 V2 (one thread).
PUBLISHED_OPTICS = (
    ("d2_100k_minpts10", 2, 100_000, 10, 231.0, "Benchmark.ods TestMatrix (min_pts 10, auto-eps)"),
    ("d2_500k_minpts10", 2, 500_000, 10, 1511.0, "Benchmark.ods TestMatrix (min_pts 10, auto-eps)"),
    ("d3_100k_minpts10", 3, 100_000, 10, 376.0, "Benchmark.ods Tabelle1 row 9 (d=3, custom kd-tree, 1 thread)"),
)


def bench_optics_published(ecc, ctx):
    """OPTICS on the published benchmark's workloads through the drop-in entry (ecc_optics_f64:
    GPU eps-balls, host seed-set expansion): wall ms per call (mean of 2 laps after a warm-up,
    host points in, host ordering out) and the GPU kernels' share."""
    res = {}
    for name, dim, n, min_pts, pub_ms, src in PUBLISHED_OPTICS:
        pts = np.random.default_rng(1).random((n, dim))
        ctx.optics_f64(pts, min_pts)  # warm-up (workspace growth)
        laps = []
        for _ in range(2):
            t0 = time.perf_counter()
            order, reach = ctx.optics_f64(pts, min_pts)
            laps.append((time.perf_counter() - t0) * 1e3)
        ctx.set_timing(True)
        ctx.timing_reset()
        ctx.optics_f64(pts, min_pts)
        st = ctx.timing_report()
        ctx.set_timing(False)
        gpu_ms = sum(v["total_ms"] for v in st.values())
        ms = sum(laps) / len(laps)
        res[name] = {"points": n, "dim": dim, "min_pts": min_pts, "ms_per_call": round(ms, 2),
                     "gpu_kernels_ms": round(gpu_ms, 3), "host_expansion_and_copies_ms": round(ms - gpu_ms, 2),
                     "published_ms": pub_ms, "published_source": src,
                     "speedup_vs_published": round(pub_ms / ms, 2),
                     "undefined_reach": int((reach < 0).sum()),
                     "kernels_ms": {k: round(v["total_ms"], 3) for k, v in sorted(st.items())}}
    return res


def shard_parity(ecc, args, dist, torch, rank, world, local, W, H, I, c0, g):
    """Sharded-run correctness (rehearsal sizes): every rank recomputes the whole stream of all
    ranks on the oracle and compares its shard's corner flags, final SAE (= the single-run SAE after
    its shard) and NMS lists, the global k-means centroids, and on rank 0 the merged tracker with
    the single-run tracker; mismatches are summed over ranks."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import orc
    from parity import nms_mismatches, tracker_mismatches
    n = args.events
    xy, t, _ = ecc.gen_events(world * n, seed=1, width=W, height=H)
    o_rx, _, o_u, _ = orc.downsample_hash(xy)
    dense = np.concatenate([o_rx[w * WINDOW: w * WINDOW + o_u[w]] for w in range(len(o_u))])
    o_c, _, _ = orc.kmeans_run_xy16(dense, c0, I)
    o_flags_r, o_sae_r = orc.fast_detect(xy[:(rank + 1) * n], t[:(rank + 1) * n], W, H)
    lo = rank * n
    cap = g["cap"]
    o_out, o_cnt, _ = orc.corner_nms(xy[lo:lo + n], o_flags_r[lo:], W, H, cap=cap)
    bad = {"flags": int(np.count_nonzero(g["flags"].numpy() != o_flags_r[lo:])),
           "sae": int(np.count_nonzero(g["sae"].numpy() != o_sae_r)),
           "centroids": int(np.count_nonzero(g["c"].numpy().view(np.uint32) != o_c.view(np.uint32))),
           "nms_slices": nms_mismatches(g["nms_out"].numpy(), g["nms_cnt"].numpy(), o_out, o_cnt, cap)[0],
           "tracker": 0}
    if rank == 0 and g["tracker"] is not None:
        f_all, _ = orc.fast_detect(xy, t, W, H)
        a_out, a_cnt, _ = orc.corner_nms(xy, f_all, W, H, cap=cap)
        otr = orc.OracleTracker(ecc.tracker_cfg())
        for s in range(len(a_cnt)):
            otr.update(a_out[s * cap: s * cap + a_cnt[s]])
        bad["tracker"] = tracker_mismatches(g["tracker"][0], otr.tracks(ecc.Track), g["tracker"][1],
                                            otr.groups(ecc.Group)[0])
    vec = torch.tensor([bad[k] for k in sorted(bad)], dtype=torch.int64, device=f"cuda:{local}")
    dist.all_reduce(vec)
    tot = dict(zip(sorted(bad), vec.cpu().tolist()))
    tot["mismatches"] = int(sum(tot.values()))
    tot["events_total"] = world * n
    return tot


def cpu_leg(ecc, args, W, H, K, I, xy, t, n, c0, ctx, g):
    """CPU baseline + full-size parity.  The oracle (single-thread C++ restatement of the
    reference algorithms, oracle/oracle.cpp) runs the step's pipeline over exactly the step's
    events on this host's cores (timed: the CPU baseline); every GPU output of the step is then
    compared with it (downsample counts + representatives, k-means centroids + labels, corner
    flags + final SAE, NMS lists, and the tracker over all slices)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import orc
    from parity import nms_mismatches, tracker_mismatches, windowed_mismatches

    t0 = time.perf_counter()
    o_rx, _, o_u, o_r = orc.downsample_hash(xy)
    dense = np.concatenate([o_rx[w * WINDOW: w * WINDOW + o_u[w]] for w in range(len(o_u))])
    o_c, o_lab, _ = orc.kmeans_run_xy16(dense, c0, I)
    o_flags, o_sae = orc.fast_detect(xy, t, W, H)
    o_out, o_cnt, _ = orc.corner_nms(xy, o_flags, W, H, cap=g["cap"])
    dt = time.perf_counter() - t0
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = platform.processor()
    base = {"value": round(n / dt / 1e6, 3), "unit": "Mevents/s", "cores": 1, "kind": "port",
            "sample": f"the step's full batch: {n} events, same pipeline (oracle/oracle.cpp, 1 thread, "
                      f"downsample + k-means + SAE/arc + NMS); {dt:.2f} s; host {model}, nproc={os.cpu_count()}"}

    # all-cores variant (oracle/cpu_omp.cpp): same pipeline, the parallel stages over every host
    # thread (OMP_NUM_THREADS); its outputs must equal the 1-thread oracle's
    nt = orc.omp_threads()
    t0 = time.perf_counter()
    p_rx, _, p_u, p_r = orc.omp_downsample_hash(xy)
    p_dense = np.concatenate([p_rx[w * WINDOW: w * WINDOW + p_u[w]] for w in range(len(p_u))])
    p_c, p_lab, _ = orc.omp_kmeans_run_xy16(p_dense, c0, I)
    p_flags, p_sae = orc.omp_fast_detect(xy, t, W, H)
    p_out, p_cnt, _ = orc.omp_corner_nms(xy, p_flags, W, H, cap=g["cap"])
    dt_omp = time.perf_counter() - t0
    omp_same = bool(np.array_equal(p_u, o_u) and np.array_equal(p_r, o_r) and np.array_equal(p_dense, dense)
                    and np.array_equal(p_c.view(np.uint32), o_c.view(np.uint32)) and np.array_equal(p_lab, o_lab)
                    and np.array_equal(p_flags, o_flags) and np.array_equal(p_sae, o_sae)
                    and np.array_equal(p_cnt, o_cnt) and nms_mismatches(p_out, p_cnt, o_out, o_cnt, g["cap"])[0] == 0)
    # the threads it may use: the job's CPU affinity and OMP_NUM_THREADS (the GPU box sets 16 for a
    # share of a larger host), not the machine's core count
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = None
    base["omp_threads"] = {
        "value": round(n / dt_omp / 1e6, 3), "unit": "Mevents/s", "cores": nt, "kind": "port",
        "equals_single_thread": omp_same,
        "limit": {"omp_threads": nt, "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
                  "affinity_cpus": aff, "host_cpus": os.cpu_count()},
        "sample": f"same {n} events and pipeline, oracle/cpu_omp.cpp (OpenMP, {nt} threads: windows, k-means "
                  f"assignment, per-slice arc tests, per-slice NMS in parallel; SAE update sequential); {dt_omp:.2f} s"}

    par = {"events": n}
    u, r = g["uniq"].numpy(), g["rep"].numpy()
    par["downsample_windows_mismatch"] = int(np.count_nonzero(u != o_u) + np.count_nonzero(r != o_r))
    par["downsample_reps_mismatch"] = windowed_mismatches(g["rep_xy"].numpy(), o_rx, o_u, WINDOW)
    gc = g["c"].numpy()
    par["kmeans_centroids_mismatch"] = int(np.count_nonzero(gc.view(np.uint32) != o_c.view(np.uint32)))
    gl = g["labels"].numpy()
    g_dense = np.concatenate([gl[w * WINDOW: w * WINDOW + o_u[w]] for w in range(len(o_u))])
    par["kmeans_labels_mismatch"] = int(np.count_nonzero(g_dense != o_lab))
    par["corner_flags_mismatch"] = int(np.count_nonzero(g["flags"].numpy() != o_flags))
    par["corner_flags_set"] = int(o_flags.sum())
    par["sae_mismatch"] = int(np.count_nonzero(g["sae"].numpy() != o_sae))
    bad, total = nms_mismatches(g["nms_out"].numpy(), g["nms_cnt"].numpy(), o_out, o_cnt, g["cap"])
    par["nms_slices_mismatch"] = bad
    par["nms_corners"] = total
    if g["tracker"] is not None:
        t1 = time.perf_counter()
        otr = orc.OracleTracker(ecc.tracker_cfg())
        for s in range(len(o_cnt)):
            otr.update(o_out[s * g["cap"]: s * g["cap"] + o_cnt[s]])
        trk_s = time.perf_counter() - t1
        o_tracks, o_groups = otr.tracks(ecc.Track), otr.groups(ecc.Group)[0]
        par["tracker_mismatch"] = tracker_mismatches(g["tracker"][0], o_tracks, g["tracker"][1], o_groups)
        par["tracker_tracks"] = len(o_tracks)
        base["tracker_us_per_slice_cpu"] = round(trk_s * 1e6 / len(o_cnt), 2)
    par["mismatches"] = int(sum(v for k, v in par.items() if k.endswith("_mismatch")))
    return base, par


if __name__ == "__main__":
    main()
