#!/bin/bash
# Phase-1 shape A/B (SRT_FW_P1_ROWS): parity for each shape, then 1-GPU C3
# and emulated N-rank timings, then a kernel trace of the emulated run.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-p1}
N=${2:-8}
mkdir -p $O
cd $R
for r in 4 2; do
  SRT_FW_P1_ROWS=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_apsp.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > $O/pytest_r$r.txt 2>&1
  rc=$?; echo "rows=$r $(tail -1 $O/pytest_r$r.txt)"; [ $rc -eq 0 ] || exit $rc
done
run() {  # tag, emu, env...
  local tag=$1 emu=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --emulate-ranks $emu > $O/$tag.json 2>&1 || return 1
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'],2), d.get('roofline',{}).get('frac'))"
}
for emu in $N 1; do
  for r in 8 4 2; do run e${emu}_r$r $emu SRT_FW_P1_ROWS=$r || exit 1; done
done
cd /tmp
for r in 4 2; do
SRT_FW_P1_ROWS=$r timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr$r -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --emulate-ranks $N > $O/trace_log$r.txt 2>&1 || exit 1
done
echo traced
