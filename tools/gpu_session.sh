#!/bin/bash
# one GPU session of round-4 work (edited per session)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4_tests29.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r4_tests29.log
bash tools/ab_c4.sh "X=1"
timeout -k 10 300 python3 bench.py --config c3ns --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-cold > gpurun_out/r4_c3ns.json 2>/dev/null; python3 -c "import json; d=json.loads(open('gpurun_out/r4_c3ns.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config']['phases_last_build'])"
