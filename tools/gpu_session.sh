#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s54
for v in 1 2; do
SRT_PKT_DRAW=$v timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_packet.py > gpurun_out/s54/t$v.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/s54/t$v.log; exit 1; }
tail -1 gpurun_out/s54/t$v.log
done
for v in 0 1 2 0 1 2; do
SRT_PKT_DRAW=$v timeout -k 10 300 python3 -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/s54/v$v.json 2> gpurun_out/s54/v$v.err || { echo "bench $v failed"; tail -5 gpurun_out/s54/v$v.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s54/v$v.json').read().strip().splitlines()[-1]); print('draw $v', d['ms_per_step'], d['roofline'].get('device_ms_per_round'))"
done
SRT_BENCH_NO_COUNTERS=1 timeout -k 10 300 python3 -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/s54/nc.json 2> gpurun_out/s54/nc.err || { echo "bench nc failed"; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s54/nc.json').read().strip().splitlines()[-1]); print('nocounters', d['ms_per_step'], d['roofline'].get('device_ms_per_round'))"
