#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a 4k build.
export TMPDIR=/tmp; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $R/gpurun_out/pmc1 -o run --output-format csv -- python3 $R/bench.py --nodes 4096 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc1.log 2>&1; echo pmc1 rc=$?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/pmc2 -o run --output-format csv -- python3 $R/bench.py --nodes 4096 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc2.log 2>&1; echo pmc2 rc=$?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc3 -o run --output-format csv -- python3 $R/bench.py --nodes 4096 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc3.log 2>&1; echo pmc3 rc=$?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc4 -o run --output-format csv -- python3 $R/bench.py --nodes 4096 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc4.log 2>&1; echo pmc4 rc=$?
ls $R/gpurun_out/pmc1
