#!/bin/bash
# Dense N-rank emulation (bench.py --emulate-ranks) with CUs reserved for the
# look-ahead chain (SRT_FW_CHAIN_CUS), then a kernel trace of the default.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-chaincus}
N=${2:-8}
mkdir -p $O
cd $R
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --emulate-ranks $N > $O/$tag.json 2>&1 || return 1
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'],2))"
}
run base SRT_X=0 || exit 1
for c in ${CUS:-8 16 32}; do
  run c$c SRT_FW_CHAIN_CUS=$c || exit 1
  run c${c}s SRT_FW_CHAIN_CUS=$c SRT_FW_CHAIN_CU_STRIDE=1 || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --emulate-ranks $N > $O/trace_log.txt 2>&1
echo "trace rc=$?"
