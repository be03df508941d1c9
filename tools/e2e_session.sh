#!/bin/bash
# End-to-end (host CSR -> host table) check: dense parity tests, then the C3
# e2e trace for the given knob sets.  Measurement / validation tool.
#   usage (GPU box): bash tools/e2e_session.sh OUT [knob sets...]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-e2e}
shift
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_apsp.py tests/test_gpu_c_abi.py tests/test_gpu_sssp.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/e2e_trace.py 16384 "$@" > $O/out.txt 2>&1; rc=$?
grep "e2e best\|create: device\|device build" $O/out.txt | tail -14
exit $rc
