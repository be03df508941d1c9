#!/bin/bash
# One GPU session: GPU tests, 4k/16k bench lines, rocprof kernel stats (4k).
export TMPDIR=/tmp; mkdir -p gpurun_out
(timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1) ; tail -3 gpurun_out/pytest_gpu.txt
(timeout -k 10 300 python -u bench.py --nodes 4096 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench4k.txt 2>&1); tail -1 gpurun_out/bench4k.txt
(timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench16k.txt 2>&1); tail -1 gpurun_out/bench16k.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4k -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --nodes 4096 --steps 1 --warmup 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof4k.log 2>&1; echo prof rc=$?
