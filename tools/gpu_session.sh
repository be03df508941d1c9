#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s33
timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_c_abi.py > gpurun_out/s33/tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/s33/tests.log; exit 1; }
tail -1 gpurun_out/s33/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
