#!/bin/bash
# round-6 session 42: the u16-unit adjacency copy for the class-CSR passes of symmetric level plans --
# level parity, then a same-box A/B against SRT_LAT16=0 on C3 and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6l16
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_local.py tests/test_gpu_configs.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for V in l16 u64 l16b u64b; do
  case $V in u64*) export SRT_LAT16=0;; *) unset SRT_LAT16;; esac
  for C in c3 c2; do
    timeout -k 10 300 python3 -u bench.py --config $C --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-cold > $O/${C}_$V.json 2> $O/${C}_$V.err || { tail -20 $O/${C}_$V.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${C}_$V.json').read().strip().splitlines()[-1]); print('$V $C', round(d['ms_per_step'],4), d['config'].get('create_device_ms'))"
  done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$O/kt.log 2>&1) || { echo "rocprof failed"; tail -5 $O/kt.log; exit 1; }
python3 -c "
import csv,sys,glob
for r in csv.DictReader(open(glob.glob('$O/kt/**/*kernel_stats.csv', recursive=True)[0])):
    if float(r['AverageNs'])>50000: print('  ', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
rm -f $(find $O -name '*kernel_trace.csv')
