#!/bin/bash
# round-6 session 4: packet tests (new round kernel), C3 bench (create spans), C3 kernel trace, C5 profile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_packet.py tests/test_golden.py tests/test_gpu_level.py tests/test_gpu_routing_info.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cold --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { echo "c3 bench failed"; tail -20 $O/c3.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$O/kt.log 2>&1) || { echo "rocprof failed"; tail -5 $O/kt.log; exit 1; }
bash tools/profile_round.sh r06c5b --config c5 --steps 50 --warmup 5 || exit 1
