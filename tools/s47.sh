#!/bin/bash
# round-6 session 47: in-process multi-GPU routing-info, rank 0 share emulated on one GPU (current code)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_multi4
timeout -k 10 600 python3 -u tools/multi_emulate.py 1 2 4 8 > gpurun_out/r06_multi4/emulated_routing_info.json 2> gpurun_out/r06_multi4/emu.err || { tail -20 gpurun_out/r06_multi4/emu.err; exit 1; }
cat gpurun_out/r06_multi4/emulated_routing_info.json | cut -c1-300
