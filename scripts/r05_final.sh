#!/bin/bash
# Round-end check at HEAD: __graft_entry__.smoke() on cuda:0, then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="$1"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
head -c 400 gpurun_out/${TAG}_bench.json
