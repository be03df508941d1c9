#!/bin/bash
# one GPU session of round-4 work (edited per session)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4_tests26.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r4_tests26.log
bash tools/ab_c3.sh "X=1" "X=2"
