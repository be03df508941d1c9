#!/bin/bash
# one GPU session of round-4 work (edited per session)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/final
for cfg in c1 c2 c2nc; do
  timeout -k 10 300 python3 bench.py --config $cfg > gpurun_out/final/r04${cfg}_bench.json 2> gpurun_out/final/$cfg.err || { echo "$cfg failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/final/r04${cfg}_bench.json').read().strip().splitlines()[-1]); print('$cfg', round(d['ms_per_step'],3), d['value'])"
done
