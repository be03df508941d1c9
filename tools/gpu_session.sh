#!/bin/bash
# one GPU session of round-4 work (edited per session)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_routing_info.py -m gpu > gpurun_out/r4_tests34.log 2>&1; echo "ri tests rc=$?"; tail -2 gpurun_out/r4_tests34.log
