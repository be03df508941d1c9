#!/bin/bash
# rocprofv3 kernel trace of a one-group C4 sparse build (per-sweep durations).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-trace_c4}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/bench.py --config c4 --in-use ${2:-192} --steps 1 --warmup 0 --no-cpu-baseline > $O/log.txt 2>&1
echo "rc=$?"; tail -2 $O/log.txt | cut -c1-300
find $O -name "*kernel_trace.csv" | head
