#!/bin/bash
# round-6 session 15: lane-group shapes of the pipelined walk (SRT_LVL_SPG: 0 = 4 lanes x 4 pairs, 1 = 4x2, 2 = 8x2, 3 = 2x4, 4 = 2x2)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6spg
mkdir -p $O
export TMPDIR=/tmp
for G in 0 1 2 3 4 0; do
  export SRT_LVL_SPG=$G
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/c3_$G.json 2> $O/c3_$G.err || { echo "bench $G failed"; tail -20 $O/c3_$G.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$G.json').read().strip().splitlines()[-1]); print('spg $G', d['ms_per_step'], d['config']['phases_last_build']['dominant_ms'])"
done
