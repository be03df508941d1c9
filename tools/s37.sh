#!/bin/bash
# round-6 session 37: staged out-rows pass, 4 vs 8 chunks in flight a lane: step times and kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6u8
mkdir -p $O
export TMPDIR=/tmp
for V in u4 u8 u4b u8b; do
  case $V in u8*) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_alt.so;; *) unset SRT_LIB;; esac
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-cold > $O/c3_$V.json 2> $O/c3_$V.err || { tail -20 $O/c3_$V.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$V.json').read().strip().splitlines()[-1]); print('$V', round(d['ms_per_step'],4))"
done
for V in u4 u8; do
  case $V in u8*) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_alt.so;; *) unset SRT_LIB;; esac
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt$V -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$O/kt$V.log 2>&1) || { echo "rocprof failed"; tail -5 $O/kt$V.log; exit 1; }
  f=$(find $O/kt$V -name '*kernel_stats.csv')
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r['AverageNs'])>50000: print('  $V', r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3)
" $f
done
rm -f $(find $O -name '*kernel_trace.csv')
