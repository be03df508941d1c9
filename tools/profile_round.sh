#!/bin/bash
# Round profile: default bench (JSON line), rocprofv3 kernel-trace stats of the
# same command, and HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE separately).
# usage: bash tools/profile_round.sh rNN
set -o pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; echo "bench rc=$?"
tail -1 $O/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py > $O/trace.log 2>&1; echo "trace rc=$?"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch.log 2>&1; echo "fetch rc=$?"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write.log 2>&1; echo "write rc=$?"
ls -R $O | head -30
