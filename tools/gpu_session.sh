#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s53
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_sssp.py tests/test_gpu_configs.py tests/test_gpu_local.py -k "sssp or c4 or sparse or frontier" > gpurun_out/s53/t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/s53/t.log; exit 1; }
tail -2 gpurun_out/s53/t.log
for v in new head new head; do
lib=$GRAFT_REPO_ROOT/shadow_amd/libsrt.so; [ $v = head ] && lib=$GRAFT_REPO_ROOT/tools/diag/libsrt_head.so
SRT_LIB=$lib timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-cold > gpurun_out/s53/$v.json 2> gpurun_out/s53/$v.err || { echo "bench $v failed"; tail -5 gpurun_out/s53/$v.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s53/$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline'].get('sweeps_per_launch'))"
done
