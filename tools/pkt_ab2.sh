#!/bin/bash
# Packet stage: tests, then C5 with/without per-pair counters, and a kernel trace.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-pkt2}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_packet.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for v in base nocount; do
  if [ $v = nocount ]; then export SRT_BENCH_NO_COUNTERS=1; fi
  timeout -k 10 200 python -u bench.py --config c5 --steps 50 --warmup 3 --no-cpu-baseline > $O/c5_$v.json 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step']*1e3,1), 'us/round wall', round(d['roofline']['device_ms_per_round']*1e3,1), 'us device')"
done
unset SRT_BENCH_NO_COUNTERS
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline > $O/trace_log.txt 2>&1
echo "trace rc=$?"
