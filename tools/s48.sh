#!/bin/bash
# round-6 session 48: the loss sweeps over reused P rows (small BA graphs, one block a launch), every sweep mode
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6reuse
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sssp.py -k "reused_rows" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
grep -cE "PASSED" $O/t.log; tail -1 $O/t.log
