#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s58
timeout -k 10 1000 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/s58/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/s58/gpu_tests.log; exit 1; }
tail -1 gpurun_out/s58/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s58/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/s58/smoke.log; exit 1; }
tail -1 gpurun_out/s58/smoke.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/s58/c3.json 2> gpurun_out/s58/c3.err || { echo "bench c3 failed"; tail -5 gpurun_out/s58/c3.err; exit 1; }
tail -1 gpurun_out/s58/c3.json | cut -c1-250
timeout -k 10 300 python3 -u bench.py --config c2 > gpurun_out/s58/c2.json 2> gpurun_out/s58/c2.err || { echo "bench c2 failed"; tail -5 gpurun_out/s58/c2.err; exit 1; }
tail -1 gpurun_out/s58/c2.json | cut -c1-250
