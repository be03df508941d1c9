#!/bin/bash
# round-6 session 53: level solve rows dealt by a self-resetting counter -- level/config/local/local-scale/auto/
# routing-info tests, then a same-box A/B against SRT_LVL_DYN=0 (static rows) on C3 and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6dyn
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_local.py tests/test_gpu_local_scale.py tests/test_gpu_auto.py tests/test_gpu_routing_info.py > $O/t.log 2>&1 || { grep -E "FAILED|Error" $O/t.log | head; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for V in dyn st dyn2 st2; do
  case $V in st*) export SRT_LVL_DYN=0;; *) unset SRT_LVL_DYN;; esac
  for C in c3 c2; do
    timeout -k 10 300 python3 -u bench.py --config $C --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-cold > $O/${C}_$V.json 2> $O/${C}_$V.err || { tail -20 $O/${C}_$V.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${C}_$V.json').read().strip().splitlines()[-1]); print('$V $C', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['config'].get('create_device_ms'))"
  done
done
