#!/bin/bash
# round-6 session 43: (8 chunks in flight) the u16-unit adjacency copy for the class-CSR passes of symmetric level plans --
# level parity, then a same-box A/B against SRT_LAT16=0 on C3 and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6l16b
mkdir -p $O
export TMPDIR=/tmp
true

for V in l16 u64 l16b u64b; do
  case $V in u64*) export SRT_LAT16=0;; *) unset SRT_LAT16;; esac
  for C in c3 c2 c1; do
    timeout -k 10 300 python3 -u bench.py --config $C --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-cold > $O/${C}_$V.json 2> $O/${C}_$V.err || { tail -20 $O/${C}_$V.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${C}_$V.json').read().strip().splitlines()[-1]); print('$V $C', round(d['ms_per_step'],4), d['config'].get('create_device_ms'))"
  done
done
unset SRT_LAT16; (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$O/kt.log 2>&1) || { echo "rocprof failed"; tail -5 $O/kt.log; exit 1; }
python3 -c "
import csv,sys,glob
for r in csv.DictReader(open(glob.glob('$O/kt/**/*kernel_stats.csv', recursive=True)[0])):
    if float(r['AverageNs'])>50000: print('  ', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
rm -f $(find $O -name '*kernel_trace.csv')
