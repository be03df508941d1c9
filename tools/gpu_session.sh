#!/bin/bash
# one GPU session of round-4 work (edited per session)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4_tests30.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4_tests30.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh r04c3 --config c3
