#!/bin/bash
# round-6 profiles A: C3 (with the SQ pass), C5, C2, C2NC -- bench line + kernel trace + PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SQPMC=1 bash tools/profile_round.sh r06c3 --steps 20 --warmup 5 || exit 1
bash tools/profile_round.sh r06c5 --config c5 --steps 50 --warmup 5 || exit 1
bash tools/profile_round.sh r06c2 --config c2 --steps 20 --warmup 5 || exit 1
bash tools/profile_round.sh r06c2nc --config c2nc --steps 20 --warmup 5 || exit 1
