#!/bin/bash
# One GPU session (run through gpurun): the GPU test suite, smoke() and the
# default bench line, each under its own time limit, stopping at the first
# failure.  Results under gpurun_out/session/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/session
timeout -k 10 1000 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/session/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/session/gpu_tests.log; exit 1; }
tail -1 gpurun_out/session/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/session/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/session/smoke.log; exit 1; }
tail -1 gpurun_out/session/smoke.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/session/bench.json 2> gpurun_out/session/bench.err || { echo "bench failed"; tail -5 gpurun_out/session/bench.err; exit 1; }
tail -1 gpurun_out/session/bench.json | cut -c1-300
