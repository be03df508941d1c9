#!/bin/bash
# Round profile of one bench config: the bench JSON line (with the CPU
# baseline), rocprofv3 kernel-trace stats of the same command, and HBM-traffic
# PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, MI355X_MICROARCH.md
# HBM section).  Summarise with tools/summarize_profile.py.
# usage: bash tools/profile_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r01}
shift
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -1 $O/bench.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py "$@" --no-cpu-baseline --no-e2e --no-cold > $O/trace.log 2>&1; rc=$?
echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-cold > $O/pmc_fetch.log 2>&1; rc=$?
echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-cold > $O/pmc_write.log 2>&1; rc=$?
echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
if [ -n "$SQPMC" ]; then
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmc_sq -o run --output-format csv -- python3 $R/bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-cold > $O/pmc_sq.log 2>&1; rc=$?
  echo "sq rc=$rc"
fi
