#!/bin/bash
# round-6 session 35: C3 class out-rows pass, chunks in flight a lane (4 default, 8, 16), kernel times under rocprofv3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6u
mkdir -p $O
export TMPDIR=/tmp
for V in 4 8 16 4b; do
  case $V in 8|16) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_u$V.so;; *) unset SRT_LIB;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$V -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-cold > $O/c3_$V.json 2> $O/c3_$V.err || { tail -20 $O/c3_$V.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$V.json').read().strip().splitlines()[-1]); print('u$V', d['ms_per_step'])"
  f=$(find $O/p$V -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'lvl_out' in r['Name'] or 'level_solve' in r['Name']: print('  ', r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3)
"
done
