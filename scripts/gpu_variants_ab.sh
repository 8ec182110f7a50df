#!/bin/bash
# Headline-step A/B over library variants: lib (default) and each lib_<tag> named in $@, both
# schedules, two rounds each (no CPU leg, no side measurements).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO" && mkdir -p gpurun_out
PKG="$REPO/event-camera-clustering-and-optical-flow-estimation_amd"
ARGS="--steps 20 --warmup 5 --no-cpu --no-tracker --no-ingest --no-eps --no-c3"
for round in 1 2; do
  for v in lib "$@"; do
    for mode in "" --serial; do
      ECC_LIB="$PKG/$v/libecc.so" timeout -k 10 300 python3 bench.py $ARGS $mode > gpurun_out/v.json 2> gpurun_out/v.err || { echo "bench $v rc=$?"; tail -5 gpurun_out/v.err; exit 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/v.json').read().strip().splitlines()[-1]);s=d['stages_ms_per_step'];print('$round $v ${mode:-two-stream}', d['ms_per_step'], {k: s[k] for k in s if k.startswith('kmeans')})"
    done
  done
done
