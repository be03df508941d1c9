#!/bin/bash
# C3 build time (and its exact-loss pass) under a few settings, 3 steps each.
# usage: bash tools/ab_c3.sh "ENV=.. ENV2=.." "ENV=.." ...
R=${GRAFT_REPO_ROOT:-$PWD}
for kv in "$@"; do
  env $kv timeout -k 10 240 python3 $R/bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-cold > $R/gpurun_out/ab_c3.json 2>/dev/null || { echo "$kv: failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$R/gpurun_out/ab_c3.json').read().strip().splitlines()[-1]); p=d['config']['phases_last_build']; print('$kv', round(d['ms_per_step'],2), 'ms, loss pass', round(p['exact_loss_pass_ms'],2), 'ms, rest', round(p['dominant_ms'],2))"
done
