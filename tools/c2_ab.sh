#!/bin/bash
# C2 (4k dense, chain-bound at 1 GPU): small-chain and phase-1 shape A/B, then a trace.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-c2ab}
mkdir -p $O
cd $R
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > $O/$tag.json 2>&1 || { tail -3 $O/$tag.json; return 1; }
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'],3), 'rest', round(d['roofline']['avg_launch_ms'],4))"
}
run base SRT_X=0 || exit 1
run small SRT_FW_SMALL_CHAIN=1 || exit 1
run p1r4 SRT_FW_P1_ROWS=4 || exit 1
run small_p1r4 SRT_FW_SMALL_CHAIN=1 SRT_FW_P1_ROWS=4 || exit 1
run small_p1r2 SRT_FW_SMALL_CHAIN=1 SRT_FW_P1_ROWS=2 || exit 1
cd /tmp
SRT_FW_SMALL_CHAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline > $O/trace_log.txt 2>&1
echo "trace rc=$?"
