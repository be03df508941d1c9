#!/bin/bash
# final r05 profile rounds of the level-solve configs (bench + trace + PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
SQPMC=1 bash tools/profile_round.sh r05c3f --config c3 --steps 10 --warmup 2 || { echo "profile c3 failed"; exit 1; }
bash tools/profile_round.sh r05c3nsf --config c3ns --steps 10 --warmup 2 || { echo "profile c3ns failed"; exit 1; }
bash tools/profile_round.sh r05c2f --config c2 --steps 10 --warmup 2 || { echo "profile c2 failed"; exit 1; }
