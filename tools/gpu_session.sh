#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s25
SRT_TRACE=1 timeout -k 10 300 python3 -u tools/multi_emulate.py 1 2 4 8 > gpurun_out/s25/emu.json 2> gpurun_out/s25/emu.err || { echo "emulate failed"; tail -5 gpurun_out/s25/emu.err; exit 1; }
cat gpurun_out/s25/emu.json | cut -c1-200
grep "multi:" gpurun_out/s25/emu.err | tail -6
