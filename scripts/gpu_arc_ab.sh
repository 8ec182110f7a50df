#!/bin/bash
# Corner parity tests on lib_exp, then the headline-step A/B (lib vs lib_exp) in both schedules.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO" && mkdir -p gpurun_out
PKG="$REPO/event-camera-clustering-and-optical-flow-estimation_amd"
ECC_LIB="$PKG/lib_exp/libecc.so" timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "${1:-fast_detect or arc or corner or sae or smoke}" > gpurun_out/arc_ab_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/arc_ab_pytest.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 20 --warmup 5 --no-cpu --no-tracker --no-ingest --no-eps --no-c3"
for mode in --serial ""; do
  for t in a b; do
    if [ $t = b ]; then export ECC_LIB="$PKG/lib_exp/libecc.so"; else unset ECC_LIB; fi
    timeout -k 10 300 python3 bench.py $ARGS $mode > gpurun_out/ab_$t.json 2> gpurun_out/ab_$t.err || { echo "bench $t rc=$?"; tail -5 gpurun_out/ab_$t.err; exit 1; }
  done
  unset ECC_LIB
  python3 - "${mode:-two-stream}" <<'PY'
import json, sys
for t in ("a", "b"):
    d = json.loads(open(f"gpurun_out/ab_{t}.json").read().strip().splitlines()[-1])
    s = d.get("stages_ms_per_step") or {}
    print(sys.argv[1], t, "ms_per_step", d["ms_per_step"], {k: s[k] for k in s if k.startswith(("arc", "pair", "slice", "flags", "sae"))})
PY
done
