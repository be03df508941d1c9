#!/bin/bash
# round-6 session 16: class CSRs from u16 latency units -- level parity, C3 bench, rank share 8, e2e trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6l16
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_local.py tests/test_gpu_local_scale.py -m gpu > $O/t0.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/t0.log | head -20; tail -30 $O/t0.log; exit 1; }
tail -1 $O/t0.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['config']['phases_last_build'], d['config'].get('create_device_ms'), d['config'].get('fresh_graph'))"
timeout -k 10 300 python3 -u bench.py --rank-share 8 --steps 20 --warmup 3 > $O/rank_share_8.json 2> $O/rank_share_8.err || { tail -20 $O/rank_share_8.err; exit 1; }
tail -1 $O/rank_share_8.json | cut -c1-600
timeout -k 10 300 python3 -u tools/ri_trace.py 16384 init > $O/ri.out 2> $O/ri.err || { tail -20 $O/ri.err; exit 1; }
cat $O/ri.out
