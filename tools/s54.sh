#!/bin/bash
# round-6 session 54: final C3 profile (dynamic row deal)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SQPMC=1 bash tools/profile_round.sh r06c3j --steps 20 --warmup 5 || exit 1
tail -1 gpurun_out/r06c3j/bench.json | cut -c1-400
