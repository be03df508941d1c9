#!/bin/bash
# Per-sweep kernel durations of one C4 sweep launch (100k BA graph, 8,192 of
# its nodes in use = one launch of 32 groups x 256 sources) for a few knob
# settings, plus a FETCH_SIZE pass of the default.  Measurement tool.
#   usage (GPU box): bash tools/c4_sweeps.sh [out-subdir] [in-use]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-c4sweeps}
N=${2:-8192}
mkdir -p $O
cd /tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 rocprofv3 --kernel-trace -d $O/$name -o run --output-format csv -- \
    python3 $R/bench.py --config c4 --in-use $N --steps 1 --warmup 0 --no-cpu-baseline > $O/$name.log 2>&1 || return 1
  python3 $R/tools/sweep_times.py $O/$name > $O/$name.txt && head -3 $O/$name.txt
}
for cfg in ${CFGS:-"fused" "split SRT_SSSP_SPLIT=1"}; do
  set -- $cfg
  run "$@" || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o run --output-format csv -- \
  python3 $R/bench.py --config c4 --in-use $N --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc.log 2>&1 || exit 1
python3 $R/tools/sweep_times.py $O/pmc --pmc FETCH_SIZE > $O/pmc.txt; head -5 $O/pmc.txt
