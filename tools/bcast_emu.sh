#!/bin/bash
# Emulated N-rank dense schedule with a stand-in for the per-round pivot-row
# broadcast latency (SRT_FW_EMU_BCAST_US) and optional chain CU reservation.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-bemu}
N=${2:-8}
mkdir -p $O
cd $R
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --emulate-ranks $N > $O/$tag.json 2>&1 || return 1
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'],2))"
}
for us in ${BCAST:-0 60 120 180}; do
  run b$us SRT_FW_EMU_BCAST_US=$us || exit 1
  for c in ${CUS:-}; do run b${us}_c$c SRT_FW_EMU_BCAST_US=$us SRT_FW_CHAIN_CUS=$c || exit 1; done
done
if [ -n "$TRACE" ]; then
cd /tmp
SRT_FW_EMU_BCAST_US=$TRACE timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --emulate-ranks $N > $O/trace_log.txt 2>&1
echo "trace rc=$?"
fi
