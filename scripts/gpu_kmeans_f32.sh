#!/bin/bash
# C3 f32 engines on the GPU: the engine parity tests, then a rocprofv3 kernel trace of the probe
# (k=16, 50 M points, 10 passes + labels) per engine.  Usage: gpu_kmeans_f32.sh <tag> [pytest -k expr]
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-km}"; KEXPR="${2:-kmeans_f32 or kmeans_c3 or kmeans_assign}"
OUT="$REPO/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest -m gpu -x -v -rf --timeout 200 --timeout-method thread -k "$KEXPR" tests/test_gpu_parity.py > "$OUT/pytest.log" 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" "$OUT/pytest.log" | tail -15
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
cd /tmp && export TMPDIR=/tmp
for e in 3 2 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/eng$e" -o p --output-format csv -- python3 "$REPO/scripts/kmeans_f32_probe.py" $e > "$OUT/eng$e.out" 2>&1 || { echo "probe $e failed"; exit 1; }
  f=$(find "$OUT/eng$e" -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -8
done
