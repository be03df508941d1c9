#!/bin/bash
# Sparse-sweep knob scan (C4 graph, 2048 in-use sources) + FW PMC pass (C3).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-tune}
mkdir -p $O
cd $R
for cfg in "1 192" "1 64" "1 600" "2 192" "2 600" "4 600"; do
  set -- $cfg
  SRT_SSSP_R=$1 SRT_SSSP_MB=$2 timeout -k 10 120 python -u bench.py --config c4 --in-use 2048 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4_R$1_MB$2.json 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('$O/c4_R$1_MB$2.json').read().strip().splitlines()[-1]); print('R=$1 MB=$2', round(d['ms_per_step'],1), d['config']['plan'])"
done
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_fw -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fw.log 2>&1; echo "pmc rc=$?"
