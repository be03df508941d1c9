#!/bin/bash
# C4 build time under a few frontier knob settings (one bench step each).
# usage: bash tools/ab_c4.sh "ENV=.. ENV2=.." "ENV=.." ...
R=${GRAFT_REPO_ROOT:-$PWD}
for kv in "$@"; do
  env $kv timeout -k 10 240 python3 $R/bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-cold > $R/gpurun_out/ab_c4.json 2>/dev/null || { echo "$kv: failed"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$R/gpurun_out/ab_c4.json').read().strip().splitlines()[-1]); print('$kv', round(d['ms_per_step'],1), 'ms', d['config']['plan'][-60:])"
done
