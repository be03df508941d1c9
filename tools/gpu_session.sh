#!/bin/bash
# one GPU session of round-5 work (edited per session)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_level.py > gpurun_out/s14_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/s14_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/s14_tests.log
SRT_TRACE=1 timeout -k 10 300 python3 -u bench.py --config c3ns --steps 5 --warmup 1 > gpurun_out/s14_c3ns.json 2> gpurun_out/s14_c3ns.err || { echo "bench failed"; tail -20 gpurun_out/s14_c3ns.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s14_c3ns.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config'].get('desc', '')[:150]); print(d['roofline'].get('avg_launch_ms'), d['roofline'].get('frac'), d['roofline'].get('edge_visits_per_row'))"
grep "level probe" gpurun_out/s14_c3ns.err | head -4
