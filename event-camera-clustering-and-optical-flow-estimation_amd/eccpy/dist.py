"""Multi-GPU time-window sharding of the event stream.

One process per GPU.  Rank r owns events [r*n, (r+1)*n) of the stream.  The exchanges:
  * k-means (bench.py): ONE all-reduce (SUM) of the shards' per-pixel count images, then every
    rank runs the Lloyd passes locally over the summed image (global_kmeans_counts) -> the
    same integer sums, hence identical centroids on all ranks, bit-identical to single-GPU;
    the per-iteration form (all-reduce of the partial sums every pass, global_kmeans) is kept
    for points that are not pixel coordinates;
  * SAE hand-off: the shards' local final time surfaces are all-gathered and rank r starts from
    the element-wise max over ranks < r (time is non-decreasing across shards, so max == last
    writer) -> corner flags identical to the single-GPU run; only rank 0 skips the first slice.
Downsample, detection and NMS are shard-local.  The tracker is sequential over slices, so the
shards' per-slice NMS lists are gathered in global slice order (gather_corner_lists: the packed
lists of every rank, all-gathered, plus each slice's start and count) and ONE tracker on rank 0
consumes them (the track merge of BASELINE config C5; reference slice path NMS -> tracker,
FCT/metavision_time_surface_periodic_group_track.cpp:832-850).

The functions here are transport- and compute-agnostic: `comm` wraps torch.distributed (RCCL on
GPUs, gloo in the CPU tests) and the compute callables are libecc on the GPU (bench.py) or the
oracle in tests/test_dist.py.
"""
from __future__ import annotations

from typing import Callable


def shard_bounds(n_total: int, world: int, rank: int, align: int = 16384) -> tuple[int, int]:
    """Contiguous time windows; every boundary is a multiple of `align` (the corner slice, which
    is also a multiple of the 8192-event downsample window), so shard-local slices are global
    slices; the last rank takes the remainder."""
    per = (n_total // world) // align * align
    lo = rank * per
    hi = n_total if rank == world - 1 else lo + per
    return lo, hi


def gather_corner_lists(comm, packed, counts):
    """Track-merge exchange.  packed: this rank's int32 tensor [T_r, 3] of kept corners (x, y,
    label), slice after slice (ecc_corner_pack); counts: int32 [ns_r] corners per slice.  Ranks
    hold consecutive time windows, so rank order is global slice order.  Returns, on every rank,
    (corners [world * T_max, 3] int32, starts int64 [sum ns_r], counts int32 [sum ns_r]): slice s
    of the global order is corners[starts[s] : starts[s] + counts[s]].  Two all-gathers (sizes,
    then the lists padded to the largest rank's); a few MB per rank at BASELINE C5."""
    import torch
    dev = packed.device
    world = comm.world
    meta = torch.tensor([packed.shape[0], counts.shape[0]], dtype=torch.int64, device=dev)
    metas = torch.zeros(world * 2, dtype=torch.int64, device=dev)
    comm.allgather_cat(metas, meta)
    sizes = metas.view(world, 2).cpu().tolist()
    t_max = max(1, max(t for t, _ in sizes))
    ns_max = max(1, max(n for _, n in sizes))
    pk = torch.zeros((t_max, 3), dtype=torch.int32, device=dev)
    pk[:packed.shape[0]] = packed
    ct = torch.zeros(ns_max, dtype=torch.int32, device=dev)
    ct[:counts.shape[0]] = counts
    all_pk = torch.zeros((world * t_max, 3), dtype=torch.int32, device=dev)
    all_ct = torch.zeros(world * ns_max, dtype=torch.int32, device=dev)
    comm.allgather_cat(all_pk.view(-1), pk.view(-1))
    comm.allgather_cat(all_ct, ct)
    starts, cnts = [], []
    for r, (_, ns) in enumerate(sizes):
        c = all_ct[r * ns_max: r * ns_max + ns].to(torch.int64)
        starts.append(r * t_max + torch.cumsum(c, 0) - c)
        cnts.append(all_ct[r * ns_max: r * ns_max + ns])
    return all_pk, torch.cat(starts), torch.cat(cnts).to(torch.int32)


class TorchComm:
    """torch.distributed transport (backend chosen at init_process_group)."""

    def __init__(self, dist):
        self.dist = dist
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()

    def allreduce_sum(self, tensor):
        self.dist.all_reduce(tensor, op=self.dist.ReduceOp.SUM)

    def allgather_cat(self, out_tensor, in_tensor):
        """out_tensor: [world * numel] contiguous; rank i's in_tensor lands at slot i."""
        self.dist.all_gather_into_tensor(out_tensor, in_tensor)

    def barrier(self):
        self.dist.barrier()


def global_kmeans(accumulate: Callable[[], object], allreduce: Callable[[object], None],
                  update: Callable[[object], bool], max_iters: int) -> int:
    """Lloyd iterations over sharded points.  accumulate() returns this rank's partial sums
    (zeroed accumulator filled for the current centroids), allreduce sums them over ranks,
    update applies the step and returns True when converged (may also always return False
    when the convergence flag lives on the device).  Returns the iterations run."""
    it = 0
    for it in range(1, max_iters + 1):
        acc = accumulate()
        allreduce(acc)
        if update(acc):
            break
    return it


def global_kmeans_counts(local_counts, allreduce: Callable[[object], None], run_counts: Callable[[object], object]):
    """K-means over sharded integer points with ONE collective: local_counts is this rank's
    per-pixel count image (additive over shards); after the all-reduce every rank runs the
    Lloyd passes over the global image (run_counts) and returns its result."""
    allreduce(local_counts)
    return run_counts(local_counts)


def sae_base_for_rank(local_images_all, rank: int, combine: Callable[[object, int], object]):
    """Initial SAE of `rank` = element-wise max of the local final SAEs of ranks < rank
    (zeros for rank 0).  local_images_all: the all-gathered [world, H*W] images."""
    return combine(local_images_all, rank)
