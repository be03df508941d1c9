#!/bin/bash
# Rehearsal of the driver's 2-rank bench (C3, its default config) on a one-GPU
# box: both ranks share device 0 (SRT_BENCH_ONE_DEVICE=1), so the times are not
# a scaling number; it checks that the N-rank path runs and prints its line.
# Not C4: two ranks of its assembled 1e10-pair table (120 GB each) staged
# through one host exceed the box's host-memory cap (killed there, r06).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s60
for c in c3; do
SRT_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --config $c --steps 3 --warmup 1 > gpurun_out/s60/$c.json 2> gpurun_out/s60/$c.err || { echo "rehearsal $c failed"; tail -8 gpurun_out/s60/$c.err; exit 1; }
tail -1 gpurun_out/s60/$c.json | cut -c1-400
done
