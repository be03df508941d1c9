# kernel-trace stats of one bench config (no CPU baseline, no e2e): the
# per-kernel breakdown behind a change.  usage: bash tools/trace_session.sh TAG [bench args...]
set -o pipefail
TAG=${1:-tr}; shift
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e "$@" > $O/trace.log 2>&1; rc=$?
echo "trace rc=$rc"; tail -1 $O/trace.log | cut -c1-300
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp $f $O/kernel_stats.csv && head -25 $O/kernel_stats.csv | cut -c1-200
exit $rc
