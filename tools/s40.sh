#!/bin/bash
# round-6 final C3 profile after the staged out-rows pass (SQ pass) + rank shares
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SQPMC=1 bash tools/profile_round.sh r06c3h --steps 20 --warmup 5 || exit 1
mkdir -p gpurun_out/r06_multi3
for N in 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --rank-share $N --steps 20 --warmup 3 > gpurun_out/r06_multi3/rank_share_$N.json 2> gpurun_out/r06_multi3/rank_share_$N.err || { echo "rank share $N failed"; tail -20 gpurun_out/r06_multi3/rank_share_$N.err; exit 1; }
  tail -1 gpurun_out/r06_multi3/rank_share_$N.json | cut -c1-330
done
