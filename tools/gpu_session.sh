#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/s31
timeout -k 10 900 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_apsp.py tests/test_gpu_level.py tests/test_gpu_routing_info.py > gpurun_out/s31/tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/s31/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/s31/tests.log
SRT_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/s31/c3.json 2> gpurun_out/s31/c3.err || { echo "bench failed"; tail -5 gpurun_out/s31/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s31/c3.json').read().strip().splitlines()[-1]); e=d['config']['e2e']; print(d['value'], d['ms_per_step'], e['ms'], e['routing_info']['ms'])"
grep -E "e2e:|create: device" gpurun_out/s31/c3.err | tail -9
