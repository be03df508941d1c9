#!/bin/bash
# one GPU session of round-5 work (edited per session)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_c_abi.py > gpurun_out/s13_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/s13_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/s13_tests.log
SQPMC=1 bash tools/profile_round.sh r05c3 --config c3 --steps 10 --warmup 2 || exit 1
