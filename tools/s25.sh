#!/bin/bash
# round-6 session 25: per-level times of the level solve after the row-phase vectorisation (-DLOSS_COUNT=1 build)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6diag3
mkdir -p $O
export TMPDIR=/tmp
SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_cnt.so timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $O/cnt.json 2> $O/cnt.err || { tail -20 $O/cnt.err; exit 1; }
grep "\[srt\]" $O/cnt.err | tail -8
