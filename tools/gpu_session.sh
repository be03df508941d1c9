#!/bin/bash
# one GPU session of round-5 work (edited per session)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s11
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_dist.py -k "level" > $O/level.log 2>&1 || { echo "level failed"; grep -E "FAIL|Error" $O/level.log | tail -20; exit 1; }
tail -1 $O/level.log
for d in 0 1 2 3; do
  SRT_LVL_DIAG=$d SRT_LIB=$PWD/shadow_amd/libsrt_cnt.so timeout -k 10 300 python3 bench.py --config c3 --steps 1 --warmup 0 --no-cold --no-cpu-baseline --no-e2e > $O/c3_cnt.json 2> $O/c3_cnt_d$d.err || { echo "cnt failed"; tail -5 $O/c3_cnt_d$d.err; }
  echo "diag=$d"; grep "level 3" $O/c3_cnt_d$d.err | tail -1
done
