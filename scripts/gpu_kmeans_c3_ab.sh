#!/bin/bash
# C3 engines A/B over library variants (lib and each lib_<tag> in $@): the bench's kmeans_c3 leg
# (downsampled representatives tiled to 50 M points), kernel averages per engine.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$REPO" && mkdir -p gpurun_out
PKG="$REPO/event-camera-clustering-and-optical-flow-estimation_amd"
for v in lib "$@" lib; do
  ECC_LIB="$PKG/$v/libecc.so" timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-tracker --no-eps --no-ingest > gpurun_out/c3.json 2> gpurun_out/c3.err || { echo "bench $v rc=$?"; tail -5 gpurun_out/c3.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/c3.json').read().strip().splitlines()[-1]);c=d['kmeans_c3'];print('$v', {k: c[k]['kernels_us'] for k in ('f32_vector','f32_mfma_32x32x2')}, c['centroids_agree'])"
done
