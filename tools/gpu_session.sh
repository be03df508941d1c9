#!/bin/bash
# one GPU session of round-5 work (edited per session)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s1
timeout -k 10 60 tools/atexit_probe 0 > gpurun_out/s1/probe.log 2>&1 || { echo "probe rc=$?"; }
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_c_abi.py tests/test_gpu_routing_info.py -k "c_ or init_async" > gpurun_out/s1/cabi.log 2>&1 || { echo "cabi failed"; tail -30 gpurun_out/s1/cabi.log; }
timeout -k 10 600 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_level.py > gpurun_out/s1/level.log 2>&1 || { echo "level failed"; grep -E "PASS|FAIL|Error|error" gpurun_out/s1/level.log | tail -40; exit 1; }
tail -3 gpurun_out/s1/level.log
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_local_scale.py > gpurun_out/s1/scale.log 2>&1 || { echo "scale failed"; tail -40 gpurun_out/s1/scale.log; exit 1; }
tail -15 gpurun_out/s1/scale.log
