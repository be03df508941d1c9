#!/bin/bash
# round-6 session 28: small levels spread over several lane groups an item -- parity, C3, C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6small
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_local.py -m gpu > $O/t0.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/t0.log | head -20; tail -30 $O/t0.log; exit 1; }
tail -1 $O/t0.log
for C in c3 c2 c3; do
timeout -k 10 300 python3 -u bench.py --config $C --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/$C.json 2> $O/$C.err || { tail -20 $O/$C.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/$C.json').read().strip().splitlines()[-1]); print('$C', d['ms_per_step'], d['config']['phases_last_build']['dominant_ms'])"
done
