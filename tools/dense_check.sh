#!/bin/bash
# Dense path check after a schedule change: parity (dense GPU tests, C ABI,
# smoke), then 1-GPU C3 and emulated N-rank timings with stand-in broadcast
# latencies (SRT_FW_EMU_BCAST_US).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-dense}
N=${2:-8}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_apsp.py tests/test_gpu_dist.py tests/test_golden.py tests/test_gpu_c_abi.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
run() {  # tag, emu, env...
  local tag=$1 emu=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --emulate-ranks $emu > $O/$tag.json 2>&1 || { tail -3 $O/$tag.json; return 1; }
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'],2), d.get('roofline',{}).get('frac'))"
}
run e1 1 SRT_X=0 || exit 1
for us in ${BCAST:-0 120 180}; do run e${N}_b$us $N SRT_FW_EMU_BCAST_US=$us || exit 1; done
for n in ${MORE:-}; do run e$n $n SRT_X=0 || exit 1; done
if [ -n "$TRACE" ]; then
cd /tmp
SRT_FW_EMU_BCAST_US=$TRACE timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --emulate-ranks $N > $O/trace_log.txt 2>&1
echo "trace rc=$?"
fi
