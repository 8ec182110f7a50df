#!/bin/bash
# A/B of an environment switch on the bench: the default run against one with VAR=VALUE (two rounds),
# printing the step and the named kernels' per-step times.
#   ab_env.sh <tag> <VAR=VALUE> "<kernel> <kernel> ..." [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="$1"; SW="$2"; KS="$3"; shift 3
for round in 1 2; do
  for v in base "$SW"; do
    name=${v//=/_}
    if [ "$v" = base ]; then
      timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-ingest --no-c3 "$@" > gpurun_out/${TAG}_${name}_$round.json 2> gpurun_out/${TAG}_${name}_$round.err || { echo "bench $v rc=$?"; tail -5 gpurun_out/${TAG}_${name}_$round.err; exit 1; }
    else
      env "$v" timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-ingest --no-c3 "$@" > gpurun_out/${TAG}_${name}_$round.json 2> gpurun_out/${TAG}_${name}_$round.err || { echo "bench $v rc=$?"; tail -5 gpurun_out/${TAG}_${name}_$round.err; exit 1; }
    fi
    python3 - "$round" "$v" "gpurun_out/${TAG}_${name}_$round.json" "$KS" <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
s = d["stages_ms_per_step"]
print(sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"], {k: round(s.get(k, float("nan")) * 1e3, 1) for k in sys.argv[4].split()})
PY
  done
done
