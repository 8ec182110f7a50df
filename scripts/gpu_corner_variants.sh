#!/bin/bash
# Corner-stage kernel times (scripts/corner_probe.py: ecc_fast_detect on the bench workload, HIP
# events per kernel) for each library variant named (lib, lib_<tag>, ...), then — if lib_prof
# exists (make ARC_PROFILE=1 LIBDIR=lib_prof) — the arc kernel's phase split.
# Usage: gpu_corner_variants.sh lib lib_x ...
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO" && mkdir -p gpurun_out
PKG="$REPO/event-camera-clustering-and-optical-flow-estimation_amd"
for v in "$@"; do
  ECC_LIB="$PKG/$v/libecc.so" timeout -k 10 120 python3 scripts/corner_probe.py > "gpurun_out/probe_$v.txt" 2>&1 || { echo "probe $v rc=$?"; tail -5 "gpurun_out/probe_$v.txt"; exit 1; }
  echo "== $v"; grep -E "^total|^corners" "gpurun_out/probe_$v.txt"
done
if [ -f "$PKG/lib_prof/libecc.so" ]; then
  ECC_LIB="$PKG/lib_prof/libecc.so" timeout -k 10 120 python3 scripts/arc_probe.py > gpurun_out/arc_probe.txt 2>&1 || { echo "arc_probe rc=$?"; tail -5 gpurun_out/arc_probe.txt; exit 1; }
  cat gpurun_out/arc_probe.txt
fi
