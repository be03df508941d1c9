#!/bin/bash
# one GPU session of round-4 work (edited per session)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4_tests28.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r4_tests28.log
SRT_TRACE=1 timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4_c3e2e.json 2> gpurun_out/r4_c3e2e.trace || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r4_c3e2e.json').read().strip().splitlines()[-1]);c=d['config'];print(d['ms_per_step'], c['e2e']['ms'], c['e2e']['call_ms'], c['e2e']['routing_info']['call_ms'], c['e2e'].get('cold',{}).get('init_first_call_ms'))"
grep "fetch8:" gpurun_out/r4_c3e2e.trace | tail -2
