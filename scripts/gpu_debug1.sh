#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 120 python scripts/debug_kmeans.py > gpurun_out/debug_kmeans.log 2>&1; echo "dbg rc=$?"; cat gpurun_out/debug_kmeans.log | head -30
timeout -k 10 300 python -X faulthandler bench.py --steps 2 --warmup 1 --no-cpu --events 2000000 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err; echo "bench rc=$?"; cat gpurun_out/bench_small.json; tail -30 gpurun_out/bench_small.err
