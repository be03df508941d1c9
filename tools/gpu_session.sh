#!/bin/bash
# emulated 8 / 4 ranks under rest LDS padding (A/B)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for pad in 0 24576 40000; do
for n in 8 4; do
  SRT_FW_REST_PAD=$pad timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold --no-e2e --emulate-ranks $n > gpurun_out/emu_pad.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/emu_pad.json').read().strip().splitlines()[-1]); print('pad $pad ranks $n', round(d['ms_per_step'],2), round(d['rest_ms_per_step'],2))"
done
done
