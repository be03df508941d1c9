#!/bin/bash
# round-6 session 23: kernel trace of the C3 step (identity-row CSR kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6id_trace
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-cold > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 - <<PY
import csv,glob
f=glob.glob('$O/trace/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1))
PY
