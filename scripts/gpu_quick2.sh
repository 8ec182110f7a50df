#!/bin/bash
# Quick GPU session: full -m gpu suite (one process) then one default bench run (with the CPU leg
# and the full-size parity check).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash scripts/gpu_tests.sh "$@" || exit $?
timeout -k 10 500 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err; rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_quick.json; tail -5 gpurun_out/bench_quick.err
