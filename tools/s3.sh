#!/bin/bash
# round-6 session 3: create-time trace of C3, 2-rank rehearsal (one device), C5 profile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
SRT_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $O/c3_trace.json 2> $O/c3_trace.err || { echo "c3 trace failed"; tail -20 $O/c3_trace.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$O/kt.log 2>&1) || { echo "rocprof failed"; tail -5 $O/kt.log; exit 1; }
SRT_BENCH_ONE_DEVICE=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --config c3 --steps 3 --warmup 1 > $O/r2.json 2> $O/r2.err || { echo "rehearsal failed"; tail -20 $O/r2.err; exit 1; }
tail -1 $O/r2.json | cut -c1-300
bash tools/profile_round.sh r06c5 --config c5 --steps 50 --warmup 5 || exit 1
