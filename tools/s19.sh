#!/bin/bash
# round-6 session 19: vectorised row init / level collection / row output of the level solve -- parity, C3, diag
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6vec
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_local.py tests/test_gpu_local_scale.py -m gpu > $O/t0.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/t0.log | head -20; tail -30 $O/t0.log; exit 1; }
tail -1 $O/t0.log
for V in a b; do
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/c3$V.json 2> $O/c3$V.err || { tail -20 $O/c3$V.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c3$V.json').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['config']['phases_last_build']['dominant_ms'])"
done
