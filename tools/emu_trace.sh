#!/bin/bash
# Kernel trace of the emulated N-rank dense critical path (one GPU): per-kernel
# start/end of every chain and rest launch, to rebuild the round period.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp
for n in ${@:-8}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/emu_trace$n${EMU_TAG} -o run --output-format csv -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cold --no-e2e --emulate-ranks $n > $R/gpurun_out/emu_trace$n${EMU_TAG}.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/emu_trace$n${EMU_TAG}.log
done
