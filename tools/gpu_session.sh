#!/bin/bash
# one GPU session of round-5 work (edited per session)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_local.py tests/test_gpu_local_scale.py tests/test_gpu_level.py > $O/local.log 2>&1 || { echo "local failed"; grep -E "FAIL|Error" $O/local.log | tail -20; }
tail -1 $O/local.log
for d in 0 1 2 3; do
  SRT_LVL_DIAG=$d SRT_LIB=$PWD/shadow_amd/libsrt_cnt.so timeout -k 10 300 python3 bench.py --config c3 --steps 1 --warmup 0 --no-cold --no-cpu-baseline --no-e2e > $O/c3_cnt.json 2> $O/c3_cnt_d$d.err || { echo "cnt failed"; tail -5 $O/c3_cnt_d$d.err; }
  echo "diag=$d"; grep "level 3" $O/c3_cnt_d$d.err | tail -1
done
