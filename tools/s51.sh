#!/bin/bash
# round-6 session 51: out-rows pass from the u16 copy: 8 (default) vs 16 chunks in flight (a1), 4 vs 8 staged hits a
# lane in pass 2 (a2); C3 steps and the pass's kernel time
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6a12
mkdir -p $O
export TMPDIR=/tmp
for V in base a1 a2 base2 a1b a2b; do
  case $V in a1*) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_a1.so;; a2*) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_a2.so;; *) unset SRT_LIB;; esac
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-cold > $O/c3_$V.json 2> $O/c3_$V.err || { tail -20 $O/c3_$V.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$V.json').read().strip().splitlines()[-1]); print('$V', round(d['ms_per_step'],4), d['config'].get('create_device_ms'))"
done
for V in base a1 a2; do
  case $V in a1*) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_a1.so;; a2*) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_a2.so;; *) unset SRT_LIB;; esac
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt$V -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$O/kt$V.log 2>&1) || { echo "rocprof failed"; tail -5 $O/kt$V.log; exit 1; }
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/kt$V/**/*kernel_stats.csv', recursive=True)[0])):
    if 'lvl_out' in r['Name']: print('  $V', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
done
rm -f $(find $O -name '*kernel_trace.csv')
