#!/bin/bash
# round-4 final profiles, part B: C4 (profile), C5 (profile), C2/C2nc/C1 bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/profile_round.sh r04c4 --config c4 || exit 1
bash tools/profile_round.sh r04c5 --config c5 || exit 1
for c in c2 c2nc c1; do
  timeout -k 10 400 python3 -u bench.py --config $c > gpurun_out/r04_$c.json 2> gpurun_out/r04_$c.err; echo "$c rc=$?"; tail -1 gpurun_out/r04_$c.json | cut -c1-200
done
