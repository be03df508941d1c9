#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s26
timeout -k 10 900 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_local_scale.py > gpurun_out/s26/tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/s26/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/s26/tests.log
for c in c3 c3ns; do
timeout -k 10 300 python3 -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/s26/$c.json 2> gpurun_out/s26/$c.err || { echo "bench failed"; tail -5 gpurun_out/s26/$c.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s26/$c.json').read().strip().splitlines()[-1]); e=d['config'].get('e2e') or {}; print('$c', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'), e.get('ms'), (e.get('routing_info') or {}).get('ms'), d['config']['plan'][:120])"
done
for N in 2 4 8; do
timeout -k 10 200 python3 -u bench.py --rank-share $N --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-cold > gpurun_out/s26/share$N.json 2> gpurun_out/s26/share$N.err || { echo "share $N failed"; tail -5 gpurun_out/s26/share$N.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s26/share$N.json').read().strip().splitlines()[-1])['rank_share']; print($N, d['ms_per_step'], d['solve_ms_per_step'])"
done
