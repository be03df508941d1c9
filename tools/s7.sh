#!/bin/bash
# round-6 session 7: the whole GPU suite, rank shares, C5 counters A/B, e2e trace, level-solve counters
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_local.py -m gpu -k "corruption or peer_copies" > $O/t0.log 2>&1 || { echo "corruption tests failed"; tail -30 $O/t0.log; exit 1; }
timeout -k 10 1100 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for N in 2 4 8; do
timeout -k 10 300 python3 -u bench.py --rank-share $N --steps 20 --warmup 3 > $O/rank_share_$N.json 2> $O/rank_share_$N.err || { echo "rank share $N failed"; tail -20 $O/rank_share_$N.err; exit 1; }
tail -1 $O/rank_share_$N.json | cut -c1-200
done
SRT_BENCH_NO_COUNTERS=1 timeout -k 10 300 python3 -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline > $O/c5_nocnt.json 2> $O/c5_nocnt.err || exit 1
tail -1 $O/c5_nocnt.json | cut -c1-200
timeout -k 10 300 python3 -u tools/ri_trace.py 16384 init > $O/ri_trace.out 2> $O/ri_trace.err || exit 1
cat $O/ri_trace.out
SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_cnt.so timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $O/cnt.json 2> $O/cnt.err || exit 1
grep "\[srt\]" $O/cnt.err | tail -12
