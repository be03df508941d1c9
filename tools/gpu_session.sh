#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/s34
timeout -k 10 900 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_apsp.py > gpurun_out/s34/tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/s34/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/s34/tests.log
for c in c3 c3ns; do
timeout -k 10 300 python3 -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-cold > gpurun_out/s34/$c.json 2> gpurun_out/s34/$c.err || { echo "bench failed"; tail -5 gpurun_out/s34/$c.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s34/$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'))"
done
