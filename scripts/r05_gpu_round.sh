#!/bin/bash
# One GPU call: the -m gpu suite, then (only if green) the probes and bench variants.
# Every GPU step has its own time limit; a step that fails stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG="${1:-r05}"
fault() { case "$1" in 0) return 0;; *) echo "rc=$1 at $2, stopping"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; fault $? pytest
tail -n 2 gpurun_out/${TAG}_pytest.log
timeout -k 10 120 python scripts/tracker_probe.py > gpurun_out/${TAG}_trk.txt 2>&1; fault $? trk
tail -n 2 gpurun_out/${TAG}_trk.txt
timeout -k 10 200 python scripts/eps_probe.py time > gpurun_out/${TAG}_eps.txt 2>&1; fault $? eps
tail -n 3 gpurun_out/${TAG}_eps.txt
for cs in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-tracker --no-ingest --no-eps --no-c3 --corner-shards $cs > gpurun_out/${TAG}_cs$cs.json 2> gpurun_out/${TAG}_cs$cs.err; fault $? bench_cs$cs
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_cs$cs.json').read().strip().splitlines()[-1]);print('cs $cs', d['value'], d['ms_per_step'], d['stages_ms_per_step'].get('arc_kernel'))"
done
