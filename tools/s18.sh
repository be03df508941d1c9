#!/bin/bash
# round-6 profiles B: C3NS, C4, C1 (bench + trace + PMC), then the rank shares at 2 / 4 / 8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/profile_round.sh r06c3ns --config c3ns --steps 10 --warmup 2 || exit 1
bash tools/profile_round.sh r06c4 --config c4 --steps 5 --warmup 1 || exit 1
bash tools/profile_round.sh r06c1 --config c1 --steps 10 --warmup 2 || exit 1
mkdir -p gpurun_out/r06_multi
for N in 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --rank-share $N --steps 20 --warmup 3 > gpurun_out/r06_multi/rank_share_$N.json 2> gpurun_out/r06_multi/rank_share_$N.err || { echo "rank share $N failed"; tail -20 gpurun_out/r06_multi/rank_share_$N.err; exit 1; }
  tail -1 gpurun_out/r06_multi/rank_share_$N.json | cut -c1-300
done
