#!/bin/bash
# one GPU session of round-4 work (edited per session)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sssp.py > gpurun_out/r4_tests18.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r4_tests18.log
bash tools/ab_c4.sh "SRT_LIB=$R/shadow_amd/libsrt.so" "SRT_LIB=$R/shadow_amd/libsrt_prev.so" "SRT_LIB=$R/shadow_amd/libsrt.so" "SRT_LIB=$R/shadow_amd/libsrt_prev.so"
