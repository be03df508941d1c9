#!/bin/bash
# Dense quick check: parity (dense GPU tests), then C2 / C3 / emulated-8 timings.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-dq}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_apsp.py tests/test_gpu_dist.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
run() {  # tag, config, steps, emu, env...
  local tag=$1 cfg=$2 steps=$3 emu=$4; shift 4
  env "$@" timeout -k 10 200 python -u bench.py --config $cfg --steps $steps --warmup 2 --no-cpu-baseline --emulate-ranks $emu > $O/$tag.json 2>&1 || { tail -3 $O/$tag.json; return 1; }
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'],3), d.get('roofline',{}).get('avg_launch_ms'))"
}
run c2 c2 10 1 SRT_X=0 || exit 1
run c3 c3 3 1 SRT_X=0 || exit 1
run e8 c3 3 8 SRT_X=0 || exit 1
