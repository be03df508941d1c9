#!/bin/bash
# round-6 session 31: needed-loss upload waits for the pinned staging -- e2e tests, default bench with cold legs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6pin
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_routing_info.py tests/test_gpu_c_abi.py -m gpu > $O/t0.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/t0.log | head -20; tail -30 $O/t0.log; exit 1; }
tail -1 $O/t0.log
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); e=d['config']['e2e']; print(d['ms_per_step'], e['ms'], e['call_ms'], e['routing_info']['call_ms'], e['cold'])"
