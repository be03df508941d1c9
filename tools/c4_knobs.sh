#!/bin/bash
# Full C4 (100k BA graph, all nodes in use) under a few sweep-batching knobs.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-c4knobs}
mkdir -p $O
cd $R
for cfg in ${KNOBS:-"1 192" "1 800" "2 800" "2 1600" "4 1600"}; do
  set -- $cfg
  SRT_SSSP_R=$1 SRT_SSSP_MB=$2 timeout -k 10 200 python -u bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > $O/c4_R$1_MB$2.json 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('$O/c4_R$1_MB$2.json').read().strip().splitlines()[-1]); print('R=$1 MB=$2', round(d['ms_per_step'],1), d['config']['plan'])"
done
