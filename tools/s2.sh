#!/bin/bash
# round-6 session: packet + golden GPU tests, C3 bench line, 2-rank rehearsal (one device), C5 profile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_packet.py tests/test_golden.py tests/test_packet_events.py tests/test_gpu_level.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cold > $O/c3.json 2> $O/c3.err || { echo "c3 bench failed"; tail -20 $O/c3.err; exit 1; }
tail -1 $O/c3.json | cut -c1-300
SRT_BENCH_ONE_DEVICE=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --config c3 --steps 3 --warmup 1 > $O/r2.json 2> $O/r2.err || { echo "rehearsal failed"; tail -20 $O/r2.err; exit 1; }
tail -1 $O/r2.json | cut -c1-300
bash tools/profile_round.sh r06c5 --config c5 --steps 50 --warmup 5 || exit 1
