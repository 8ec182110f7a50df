#!/bin/bash
# A/B of the headline step: bench.py with the default libecc and with lib_exp (ECC_LIB), kernel
# averages and step time of each (no CPU leg, no side measurements).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO" && mkdir -p gpurun_out
PKG="$REPO/event-camera-clustering-and-optical-flow-estimation_amd"
ARGS="--steps 20 --warmup 5 --no-cpu --no-tracker --no-ingest --no-eps --no-c3"
timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab_a.json 2> gpurun_out/ab_a.err || exit $?
ECC_LIB="$PKG/lib_exp/libecc.so" timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab_b.json 2> gpurun_out/ab_b.err || exit $?
python3 - <<'PY'
import json
for t in ("a", "b"):
    d = json.loads(open(f"gpurun_out/ab_{t}.json").read().strip().splitlines()[-1])
    print(t, "ms_per_step", d["ms_per_step"], d.get("stages_ms_per_step"))
PY
