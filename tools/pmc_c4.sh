#!/bin/bash
# SQ / TCC / TA counter passes over one C4 sweep launch (8,192 in-use
# sources = 32 sweeps of 32 groups), one rocprofv3 run per pass.  Measurement
# tool; summarise with tools/sweep_times.py DIR --pmc COUNTER.
#   usage (GPU box): bash tools/pmc_c4.sh [out-subdir] [in-use]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-pmcc4}
N=${2:-8192}
mkdir -p $O
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
            "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
            "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  ${EXTRA_ENV:+env $EXTRA_ENV} timeout -s KILL 120 rocprofv3 --pmc $pass -d $O/p$i -o run --output-format csv -- \
    python3 $R/bench.py --config c4 --in-use $N --steps 1 --warmup 0 --no-cpu-baseline > $O/p$i.log 2>&1
  echo "pass $i rc=$?"
done
exit 0
