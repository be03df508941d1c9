#!/bin/bash
# round-6 session 52: per-build counter resets in one tiny kernel -- level / config / local / local-scale / auto /
# routing-info tests, then C3 and C2 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6zero
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_local.py tests/test_gpu_local_scale.py tests/test_gpu_auto.py tests/test_gpu_routing_info.py > $O/t.log 2>&1 || { grep -E "FAILED|Error" $O/t.log | head; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for C in c3 c2 c3ns; do
  timeout -k 10 300 python3 -u bench.py --config $C --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-cold > $O/$C.json 2> $O/$C.err || { tail -20 $O/$C.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$C.json').read().strip().splitlines()[-1]); c=d['config']; print('$C', round(d['ms_per_step'],4), c.get('create_device_ms'), c.get('plan'))"
done
