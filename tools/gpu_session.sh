#!/bin/bash
set -o pipefail
bash $GRAFT_REPO_ROOT/tools/profile_round.sh r05c2g --config c2 --steps 10 --warmup 2
