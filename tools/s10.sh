#!/bin/bash
# round-6 session 10: level-solve geometry A/B on C3 (SRT_LVL_GEOM 0..3), each checked by the level tests first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6geom
mkdir -p $O
export TMPDIR=/tmp
for G in 0 1 2 3; do
  export SRT_LVL_GEOM=$G
  timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_level.py -m gpu > $O/t$G.log 2>&1 || { echo "tests failed geom $G"; grep -E "FAILED|Error" $O/t$G.log | head -20; tail -30 $O/t$G.log; exit 1; }
  tail -1 $O/t$G.log
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/c3_$G.json 2> $O/c3_$G.err || { echo "bench $G failed"; tail -20 $O/c3_$G.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$G.json').read().strip().splitlines()[-1]); print('geom $G', d['ms_per_step'], d['config']['phases_last_build'])"
done
