#!/bin/bash
# round-6 session 39: class-ballot positions in the out-rows pass: out-rows pass with hits staged in LDS -- level parity, then a same-box A/B against the
# previous library (SRT_LIB=libsrt_alt.so) on C3, C2 and C3NS
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6mt
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_local.py tests/test_gpu_configs.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for V in new alt new2 alt2; do
  case $V in alt*) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_alt.so;; *) unset SRT_LIB;; esac
  for C in c3 c2 c3ns; do
    timeout -k 10 300 python3 -u bench.py --config $C --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-cold > $O/${C}_$V.json 2> $O/${C}_$V.err || { tail -20 $O/${C}_$V.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${C}_$V.json').read().strip().splitlines()[-1]); print('$V $C', round(d['ms_per_step'],4), d['config'].get('create_device_ms'))"
  done
done
