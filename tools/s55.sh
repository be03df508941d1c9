#!/bin/bash
# round-6 session 55: rank shares with the solve row counter
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_multi5
for N in 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --rank-share $N --steps 20 --warmup 3 > gpurun_out/r06_multi5/rank_share_$N.json 2> gpurun_out/r06_multi5/rank_share_$N.err || { echo "rank share $N failed"; tail -20 gpurun_out/r06_multi5/rank_share_$N.err; exit 1; }
  python3 -c "import json; d=json.loads(open(\"gpurun_out/r06_multi5/rank_share_$N.json\").read().strip().splitlines()[-1])[\"rank_share\"]; print($N, d[\"ms_per_step\"], d[\"solve_ms_per_step\"])"
done
