REPO="${GRAFT_REPO_ROOT}"; PKG="$REPO/event-camera-clustering-and-optical-flow-estimation_amd"; cd /tmp && export TMPDIR=/tmp
for v in lib lib_b2w4 lib_b1w6 lib_b2w6; do
  ECC_LIB="$PKG/$v/libecc.so" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/ab/$v" -o p --output-format csv -- python3 "$REPO/scripts/kmeans_f32_probe.py" 3 > "$REPO/gpurun_out/ab/$v.out" 2>&1 || { echo "$v failed"; exit 1; }
  f=$(find "$REPO/gpurun_out/ab/$v" -name "*kernel_stats.csv" | head -1); echo "$v"; cut -d, -f1-4 "$f" | grep pair_kernel | sed 's/.*kernel<16, \(true\|false\).*",\([0-9]*\),\([0-9]*\),\(.*\)/\1 \2 \4/'
done
