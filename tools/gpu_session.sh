#!/bin/bash
# one GPU session of round-4 work (edited per session)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/ab_c3.sh "SRT_LIB=$R/shadow_amd/libsrt_a.so" "SRT_LIB=$R/shadow_amd/libsrt.so" "SRT_LIB=$R/shadow_amd/libsrt_a.so" "SRT_LIB=$R/shadow_amd/libsrt.so" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_apsp.py tests/test_gpu_configs.py -m gpu -k "loss or level or c3" > gpurun_out/r4_t.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r4_t.log
