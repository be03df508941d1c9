#!/bin/bash
# round-6 session 45: symmetry check writing the u16 copy 8 B a store through the LDS tile (libsrt.so) against
# 2-B stores (libsrt_alt.so): symmetric-row tests, then C3 create device work and step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6p16
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_level.py -k "symmetric or sharded or rank" tests/test_gpu_configs.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for V in new alt new2 alt2; do
  case $V in alt*) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_alt.so;; *) unset SRT_LIB;; esac
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-cold > $O/c3_$V.json 2> $O/c3_$V.err || { tail -20 $O/c3_$V.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$V.json').read().strip().splitlines()[-1]); print('$V', round(d['ms_per_step'],4), d['config'].get('create_device_ms'))"
done
unset SRT_LIB
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$O/kt.log 2>&1) || { echo "rocprof failed"; tail -5 $O/kt.log; exit 1; }
python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/kt/**/*kernel_stats.csv', recursive=True)[0])):
    if float(r['AverageNs'])>50000: print('  ', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
rm -f $(find $O -name '*kernel_trace.csv')
