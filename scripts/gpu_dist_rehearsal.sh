#!/bin/bash
# Rehearse the sharded bench path on the 1-GPU box: 2 ranks on device 0 over gloo, small batch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 2 --warmup 1 --events $((16384*64)) --no-cpu --no-eps --no-ingest --dist-backend gloo --same-device --dist-parity \
  > gpurun_out/dist_rehearsal.json 2> gpurun_out/dist_rehearsal.err
rc=$?; echo "dist rc=$rc"; cat gpurun_out/dist_rehearsal.json; tail -20 gpurun_out/dist_rehearsal.err
