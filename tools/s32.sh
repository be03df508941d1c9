#!/bin/bash
# round-6 session 32: level probe at 15 classes first -- level/config/auto tests, C3/C2/C1 create and step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6p15
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_auto.py tests/test_gpu_local.py -m gpu > $O/t0.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/t0.log | head -20; tail -30 $O/t0.log; exit 1; }
tail -1 $O/t0.log
for C in c3 c2 c2nc c3ns; do
timeout -k 10 300 python3 -u bench.py --config $C --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/$C.json 2> $O/$C.err || { tail -20 $O/$C.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/$C.json').read().strip().splitlines()[-1]); c=d['config']; print('$C', d['ms_per_step'], c.get('create_device_ms'), (c.get('fresh_graph') or {}).get('ms'), c.get('plan'))"
done
