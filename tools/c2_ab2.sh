#!/bin/bash
# C2 after the automatic small chain: event-packet variants; C3 unchanged check.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-c2ab2}
mkdir -p $O
cd $R
run() {  # tag, config, env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $O/$tag.json 2>&1 || { tail -3 $O/$tag.json; return 1; }
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'],3), 'rest', round(d['roofline']['avg_launch_ms'],4))"
}
run c2 c2 SRT_X=0 || exit 1
run c2_ev16 c2 SRT_FW_EVENT_EVERY=16 || exit 1
run c2_sync c2 SRT_FW_SYNC_FENCE=1 || exit 1
run c2_both c2 SRT_FW_EVENT_EVERY=16 SRT_FW_SYNC_FENCE=1 || exit 1
STEPS=3 run c3 c3 SRT_X=0 || exit 1
