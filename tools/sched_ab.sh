#!/bin/bash
# Dense-schedule check: parity tests, then 1-GPU C3 and emulated N-rank
# timings under a few knobs, then a kernel trace of the emulated run.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-sched}
N=${2:-8}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_apsp.py tests/test_gpu_dist.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
run() {  # tag, emu, env...
  local tag=$1 emu=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --emulate-ranks $emu > $O/$tag.json 2>&1 || return 1
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'],2), d.get('roofline',{}).get('frac'))"
}
for emu in 1 $N; do
  run e${emu}_base $emu SRT_X=0 || exit 1
  run e${emu}_sync $emu SRT_FW_SYNC_FENCE=1 || exit 1
done
for emu in ${MORE:-}; do run e${emu}_base $emu SRT_X=0 || exit 1; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --emulate-ranks $N > $O/trace_log.txt 2>&1
echo "trace rc=$?"
