#!/bin/bash
# Round evidence in one GPU call: full -m gpu suite + smoke, rocprofv3 kernel stats + PMC traffic
# passes of the bench, then the default bench (with cpu_baseline).  Usage: gpu_round.sh <tag>
TAG="${1:-r01d}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash scripts/gpu_tests.sh || exit $?
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed" gpurun_out/pytest_gpu.log || { echo "tests failed"; exit 1; }
bash scripts/gpu_profile.sh "$TAG" || exit $?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
python3 scripts/traffic.py "gpurun_out/prof_$TAG" "gpurun_out/prof_$TAG/traffic.json" || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
echo "bench rc=$rc"; head -c 400 gpurun_out/bench_$TAG.json
