#!/bin/bash
# round-6 session 5: packet tests, C5 trace, C3 bench (create spans)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_packet.py tests/test_golden.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c5kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/c5kt.log 2>&1) || { echo "rocprof failed"; tail -5 $O/c5kt.log; exit 1; }
grep -h round_kernel $O/c5kt/run_kernel_stats.csv | cut -c1-40,200-260
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/c3.json 2> $O/c3.err || { echo "c3 bench failed"; tail -20 $O/c3.err; exit 1; }
tail -1 $O/c3.json | cut -c1-200
