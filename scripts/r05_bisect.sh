#!/bin/bash
# Runs the 1-rank RCCL sharded step with dist parity under each library variant named in $@.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
PKG=event-camera-clustering-and-optical-flow-estimation_amd
for v in "$@"; do
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + RANDOM % 300)) ECC_LIB="$PWD/$PKG/$v/libecc.so" timeout -k 10 200 \
    python3 bench.py --force-dist --dist-backend nccl --events 655360 --steps 2 --warmup 1 --no-cpu --no-eps --no-ingest --no-c3 --dist-parity \
    > gpurun_out/bis_$v.json 2> gpurun_out/bis_$v.err || { echo "$v rc=$?"; tail -5 gpurun_out/bis_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['dist_parity'])" gpurun_out/bis_$v.json $v
done
