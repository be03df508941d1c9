#!/bin/bash
# round-6 session 12: pipelined push/pull-split level walk (SRT_LVL_SP=1 default) -- level parity, C3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6sp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_local.py -m gpu > $O/t0.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/t0.log | head -20; tail -30 $O/t0.log; exit 1; }
tail -1 $O/t0.log
for V in sp1 sp0 sp1b; do
  case $V in sp0) export SRT_LVL_SP=0;; *) export SRT_LVL_SP=1;; esac
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/c3_$V.json 2> $O/c3_$V.err || { echo "bench $V failed"; tail -20 $O/c3_$V.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$V.json').read().strip().splitlines()[-1]); print('$V', d['ms_per_step'], d['config']['phases_last_build'])"
done
