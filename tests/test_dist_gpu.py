"""The sharded (C5) step of bench.py executed on the GPU through libecc — not the oracle.

* A 1-rank RCCL (`nccl`) process group (`--force-dist`): the two-stream schedule of the sharded
  step (downsample -> count image -> all-reduce issued from the k-means stream -> Lloyd passes ->
  labels, beside prepare -> all-gather -> `ecc_sae_max_combine` -> finish -> NMS), then
  `ecc_corner_pack` -> `gather_corner_lists` -> ONE `ecc_tracker_update_lists` on rank 0.
* Two gloo ranks on the one GPU with the same overlapped schedule (`--overlap`): the SAE hand-off
  between real shards and the merged tracker over two ranks' lists.

Both compare every shard output, the global centroids and the merged tracker with the oracle
over the whole stream (`--dist-parity`; reference anchor: the slice path
FCT/metavision_time_surface_periodic_group_track.cpp:832-850 that the merge restates).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, timeout=240, port=None):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env["MASTER_ADDR"] = "127.0.0.1"
    if port is not None:
        env["MASTER_PORT"] = str(port)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(lines[-1])


COMMON = ["--steps", "2", "--warmup", "1", "--no-cpu", "--no-eps", "--no-ingest", "--no-c3", "--dist-parity"]


@pytest.mark.gpu
def test_rccl_one_rank_sharded_step_matches_oracle():
    cmd = [sys.executable, "bench.py", "--force-dist", "--dist-backend", "nccl",
           "--events", str(16384 * 40)] + COMMON
    res = _run(cmd, port=_free_port())
    par = res["dist_parity"]
    assert par is not None and par["mismatches"] == 0, par
    tm = res["track_merge"]
    assert tm is not None and tm["ranks"] == 1 and tm["slices"] == 40 and tm["tracks_end"] > 0, tm
    assert tm["pipelined"]["mevents_s"] > 0 and tm["pipelined"]["steps"] >= 3, tm
    assert res["n_gpus"] == 1
    # rank 0's single-GPU rate at the same per-GPU size, measured in the same job
    n1 = res["per_gpu_rate_n1"]
    assert n1 is not None and n1["value"] > 0 and n1["events_per_gpu"] == 16384 * 40, n1


@pytest.mark.gpu
def test_gloo_two_ranks_overlapped_schedule_matches_oracle():
    """`bench.py --gpus 2` with NO external launcher: bench.py itself starts the two ranks (a
    torch.distributed.run child), and the line says so (n_gpus, dist_world)."""
    cmd = [sys.executable, "bench.py", "--gpus", "2",
           "--events", str(16384 * 24), "--dist-backend", "gloo", "--same-device", "--overlap"] + COMMON
    res = _run(cmd, timeout=300)
    assert res["n_gpus"] == 2 and res["dist_world"] == 2 and res["dist_backend"] == "gloo", res
    par = res["dist_parity"]
    assert par is not None and par["mismatches"] == 0, par
    assert par["events_total"] == 2 * 16384 * 24
    tm = res["track_merge"]
    assert tm is not None and tm["ranks"] == 2 and tm["slices"] == 48 and tm["tracks_end"] > 0, tm
    assert tm["pipelined"]["mevents_s"] > 0, tm
    assert res["config"]["events_total"] == 2 * 16384 * 24 and res["config"]["workload"].startswith("C5"), res["config"]
    assert res["per_gpu_rate_n1"]["value"] > 0
