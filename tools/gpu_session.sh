#!/bin/bash
# one GPU session of round-5 work (edited per session)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s9
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_all.log 2>&1
echo "rc=$?"
grep -E "FAILED|ERROR" $O/gpu_all.log | head -40
tail -3 $O/gpu_all.log
