#!/bin/bash
# Fresh-box validation: GPU tests, smoke(), default bench line (C3 + CPU baseline),
# C2 line, rocprofv3 kernel stats of the default bench.  Stops at the first failure.
export TMPDIR=/tmp; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 \
 && tail -3 gpurun_out/pytest_gpu.txt \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 \
 && tail -1 gpurun_out/smoke.txt \
 && timeout -k 10 400 python -u bench.py > gpurun_out/bench_c3.txt 2>&1 \
 && tail -1 gpurun_out/bench_c3.txt \
 && timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 2 > gpurun_out/bench_c2.txt 2>&1 \
 && tail -1 gpurun_out/bench_c2.txt \
 && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c3.log 2>&1 \
 && echo prof ok
