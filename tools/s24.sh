#!/bin/bash
# round-6 session 24: the whole GPU suite, smoke(), the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6full2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
