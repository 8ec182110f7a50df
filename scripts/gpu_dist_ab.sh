cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
# gloo rehearsal A/B of the two schedules: --overlap keeps the two-stream step under gloo
for a in --overlap --serial --overlap --serial; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 6 --warmup 2 --events $((16384*256)) --no-cpu --no-eps --no-ingest --no-c3 --no-tracker --dist-backend gloo --same-device $a \
  > gpurun_out/dr2.json 2> gpurun_out/dr2.err || exit 1
echo "$a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dr2.json | head -1)"
done
