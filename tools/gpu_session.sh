#!/bin/bash
# one GPU session of round-5 work (edited per session)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s17
cd /tmp
for c in c3 c3ns; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s17/$c -o run --output-format csv -- python3 $R/bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-cold > $R/gpurun_out/s17/$c.log 2>&1 || { echo "trace $c failed"; tail -5 $R/gpurun_out/s17/$c.log; exit 1; }
python3 - $R/gpurun_out/s17/$c <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:70].ljust(70), r['Calls'].rjust(5), '%.3f ms avg' % (float(r['AverageNs'])/1e6))
PY
done
