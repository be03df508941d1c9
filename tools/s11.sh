#!/bin/bash
# round-6 session 11: e2e routing_info trace, loss range check started before (A) / after (B) the needed-loss gather
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e2e2
mkdir -p $O
export TMPDIR=/tmp
for V in early late early2 late2; do
  case $V in early*) export SRT_LOSSCHK_EARLY=1;; *) export SRT_LOSSCHK_EARLY=0;; esac
  timeout -k 10 300 python3 -u tools/ri_trace.py 16384 init > $O/ri_$V.out 2> $O/ri_$V.err || { tail -20 $O/ri_$V.err; exit 1; }
  echo "== $V"; cat $O/ri_$V.out
  grep "losses: gathered\|records touched\|e2e: create\|build + fetch" $O/ri_$V.err | tail -4
done
