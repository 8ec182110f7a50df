#!/bin/bash
# Copy a gpu_round.sh / gpu_evidence.sh run's summaries from gpurun_out/ into profiles/ (tracked):
#   collect_evidence.sh <tag>
# kernel stats (+ the meta file naming the libecc it was traced with, which bench.py checks before
# it reports the rocprof average), traffic, occupancy, calibration, bench line, pytest log, and
# the DBSCAN / list-chain PMC summaries when present.
cd "$(dirname "$0")/.." || exit 1
T="$1"; E=gpurun_out/ev_$T; P=profiles
[ -d "$E" ] || { echo "no $E"; exit 1; }
cp "$(find "$E/trace" -name '*kernel_stats.csv' | head -1)" $P/${T}_kernel_stats.csv
[ -f "$E/kernel_stats.meta.json" ] && cp "$E/kernel_stats.meta.json" $P/${T}_kernel_stats.meta.json
for f in traffic.json traffic.txt occupancy.json occupancy.txt calib.txt; do [ -f "$E/$f" ] && cp "$E/$f" $P/${T}_$f; done
[ -f "$E/bench.json" ] && cp "$E/bench.json" $P/${T}_bench.json
[ -f "$E/trace_bench.json" ] && cp "$E/trace_bench.json" $P/${T}_bench_under_rocprof.json
[ -f gpurun_out/${T}_pytest.log ] && cp gpurun_out/${T}_pytest.log $P/${T}_pytest_gpu.log
for k in db lists; do
  D=gpurun_out/pmc_${k}_$T
  [ -d "$D" ] || continue
  cp "$(find "$D/trace" -name '*kernel_stats.csv' | head -1)" $P/${T}_${k}_kernel_stats.csv
  cp "$D/traffic.txt" $P/${T}_${k}_traffic.txt; cp "$D/occupancy.txt" $P/${T}_${k}_occupancy.txt
  cp "$D/occupancy.json" $P/${T}_${k}_occupancy.json
done
ls -la $P/${T}_*
