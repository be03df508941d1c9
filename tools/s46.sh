#!/bin/bash
# round-6 session 46: final C3 profile (u16 adjacency copy for the class out-rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SQPMC=1 bash tools/profile_round.sh r06c3i --steps 20 --warmup 5 || exit 1
tail -1 gpurun_out/r06c3i/bench.json | cut -c1-400
