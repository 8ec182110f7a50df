#!/bin/bash
# A/B of library variants on the bench: lib (default) and each lib_<tag> named in $@ (two rounds).
# Usage: ab_libs.sh <tag> <extra bench args...> -- <variant dirs...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="$1"; shift
ARGS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do ARGS+=("$1"); shift; done; shift
PKG=event-camera-clustering-and-optical-flow-estimation_amd
for round in 1 2; do
  for v in lib "$@"; do
    ECC_LIB="$PWD/$PKG/$v/libecc.so" timeout -k 10 400 python3 bench.py "${ARGS[@]}" > gpurun_out/${TAG}_${v}_$round.json 2> gpurun_out/${TAG}_${v}_$round.err || { echo "bench $v rc=$?"; tail -5 gpurun_out/${TAG}_${v}_$round.err; exit 1; }
    python3 - "$round" "$v" "gpurun_out/${TAG}_${v}_$round.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
s = d["stages_ms_per_step"]
eps = d.get("eps") or {}
tr = d.get("tracker") or {}
print(sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"], "arc", s.get("arc_kernel"), "dense", s.get("arc_dense_kernel"),
      "trk", tr.get("us_per_slice"), "grid", (eps.get("dbscan_grid_eps20_minpts20") or {}).get("kernels_us"),
      "chain", (eps.get("dbscan_chain_eps20_minpts20") or {}).get("ms_per_call"))
PY
  done
done
