#!/bin/bash
# Full round session: parity suite + smoke, 2-rank rehearsal, rocprofv3 (trace + PMC), bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="${1:-r01b}"
bash scripts/gpu_tests.sh || exit $?
bash scripts/gpu_dist_rehearsal.sh || exit $?
bash scripts/gpu_profile.sh "$TAG" || exit $?
python3 scripts/traffic.py "gpurun_out/prof_$TAG" "gpurun_out/${TAG}_traffic.json" > gpurun_out/traffic.txt 2>&1; cat gpurun_out/traffic.txt
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "bench rc=$?"; cat gpurun_out/bench.json
