#!/bin/bash
# round-6 session 26: flat-streamed identity-row class CSR (SRT_LVL_FLAT=1 default) -- parity, C3 A/B, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6flat
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_local.py tests/test_gpu_local_scale.py -m gpu > $O/t0.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/t0.log | head -20; tail -30 $O/t0.log; exit 1; }
tail -1 $O/t0.log
for V in f1 f0 f1b f0b; do
  case $V in f0*) export SRT_LVL_FLAT=0;; *) export SRT_LVL_FLAT=1;; esac
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/c3_$V.json 2> $O/c3_$V.err || { echo "bench $V failed"; tail -20 $O/c3_$V.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$V.json').read().strip().splitlines()[-1]); c=d['config']; print('$V', d['ms_per_step'], c['phases_last_build']['dominant_ms'], c.get('create_device_ms'))"
done
unset SRT_LVL_FLAT
timeout -k 10 300 python3 -u bench.py --rank-share 8 --steps 20 --warmup 3 > $O/rank_share_8.json 2> $O/rank_share_8.err || { tail -20 $O/rank_share_8.err; exit 1; }
tail -1 $O/rank_share_8.json | cut -c1-420
