#!/bin/bash
# Kernel trace, HBM traffic and SQ counter passes over ONE probe command, each pass under its own
# time limit (PMC passes with --kernel-trace only, never sys/runtime traces):
#   gpu_pmc.sh <tag> <python script under scripts/> [args...]
# e.g. gpu_pmc.sh lists eps_probe.py lists | gpu_pmc.sh corner corner_probe.py | gpu_pmc.sh trk tracker_probe.py
# Writes gpurun_out/pmc_<tag>/{trace,fetch,write,sq/p1,sq/p2} and the summaries traffic.txt and
# occupancy.txt (scripts/traffic.py, scripts/pmc_summary.py).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; SCRIPT="$REPO/scripts/$2"; shift 2
OUT="$REPO/gpurun_out/pmc_$TAG"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
pass() {  # pass <dir> [rocprofv3 options]
  local d="$1"; shift
  timeout -s KILL 180 rocprofv3 --kernel-trace "$@" -d "$OUT/$d" -o p --output-format csv -- python3 "$SCRIPT" $ARGS \
    > "$OUT/${d//\//_}.log" 2>&1 || { echo "pass $d rc=$?"; tail -3 "$OUT/${d//\//_}.log"; exit 1; }
}
ARGS="$*"
pass trace --stats
pass fetch --pmc FETCH_SIZE
pass write --pmc WRITE_SIZE
pass sq/p1 --pmc $P1
pass sq/p2 --pmc $P2
cd "$REPO"
python3 scripts/traffic.py "$OUT" "$OUT/traffic.json" > "$OUT/traffic.txt" || exit 1
python3 scripts/pmc_summary.py "$OUT/sq" "$OUT/occupancy.json" > "$OUT/occupancy.txt" || exit 1
cat "$OUT/traffic.txt" "$OUT/occupancy.txt"
