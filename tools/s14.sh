#!/bin/bash
# round-6 session 14: per-level walk time of the pipelined walk, with the loss atomics (diag 1), the level
# stores (2) or both (3) dropped (-DLOSS_COUNT=1 build: timing only, wrong tables)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6diag
mkdir -p $O
export TMPDIR=/tmp
for D in 0 1 2 3; do
  SRT_LVL_DIAG=$D SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_cnt.so timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $O/cnt$D.json 2> $O/cnt$D.err || { tail -20 $O/cnt$D.err; exit 1; }
  echo "== diag $D"; grep "\[srt\]" $O/cnt$D.err | tail -5
done
