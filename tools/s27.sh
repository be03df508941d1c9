#!/bin/bash
# round-6 final profiles: C3 (SQ pass), C2, C2NC, C3NS with the current level solve; the 2-rank C3 rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SQPMC=1 bash tools/profile_round.sh r06c3f --steps 20 --warmup 5 || exit 1
bash tools/profile_round.sh r06c2f --config c2 --steps 20 --warmup 5 || exit 1
bash tools/profile_round.sh r06c2ncf --config c2nc --steps 20 --warmup 5 || exit 1
bash tools/profile_round.sh r06c3nsf --config c3ns --steps 10 --warmup 2 || exit 1
mkdir -p gpurun_out/r06_reh
SRT_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --config c3 --steps 3 --warmup 1 > gpurun_out/r06_reh/c3.json 2> gpurun_out/r06_reh/c3.err || { echo "rehearsal failed"; tail -8 gpurun_out/r06_reh/c3.err; exit 1; }
tail -1 gpurun_out/r06_reh/c3.json | cut -c1-600
