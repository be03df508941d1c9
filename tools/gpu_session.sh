#!/bin/bash
# one GPU session of round-5 work (edited per session)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s5
mkdir -p $O
export TMPDIR=/tmp
for k in 0 8; do
  SRT_LVL_K=$k SRT_LIB=$PWD/shadow_amd/libsrt_cnt.so timeout -k 10 300 python3 bench.py --config c3 --steps 1 --warmup 0 --no-cold --no-cpu-baseline --no-e2e > $O/c3_cnt$k.json 2> $O/c3_cnt$k.err || { echo "cnt failed"; tail -5 $O/c3_cnt$k.err; }
  echo "K=$k"; grep "level" $O/c3_cnt$k.err | grep -v probe | tail -8
done
