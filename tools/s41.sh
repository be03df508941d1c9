#!/bin/bash
# round-6 session 41: C5 profile refresh (bench line reads the r06c5 traffic summary)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/profile_round.sh r06c5b --config c5 --steps 50 --warmup 5 || exit 1
tail -1 gpurun_out/r06c5b/bench.json | cut -c1-900
