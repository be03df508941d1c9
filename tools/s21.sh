#!/bin/bash
# round-6 session 21: the pipelined walk two chunks ahead (SRT_LVL_SP=2) vs one (1) -- parity under both, C3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6d2
mkdir -p $O
export TMPDIR=/tmp
for S in 2 1; do
  export SRT_LVL_SP=$S
  timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py -m gpu > $O/t$S.log 2>&1 || { echo "tests failed sp$S"; grep -E "FAILED|Error" $O/t$S.log | head -20; tail -30 $O/t$S.log; exit 1; }
  tail -1 $O/t$S.log
done
for V in 2 1 2b 1b; do
  export SRT_LVL_SP=${V%b}
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/c3_$V.json 2> $O/c3_$V.err || { echo "bench $V failed"; tail -20 $O/c3_$V.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$V.json').read().strip().splitlines()[-1]); print('sp$V', d['ms_per_step'], d['config']['phases_last_build']['dominant_ms'])"
done
