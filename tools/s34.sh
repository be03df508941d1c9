#!/bin/bash
# round-6 session 34: C5 round kernel, hosts a workgroup A/B (HB 16 default, 8, 32), with and without counters
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6hb
mkdir -p $O
export TMPDIR=/tmp
for V in 16 8 32 16b; do
  case $V in 8|32) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_hb$V.so;; *) unset SRT_LIB;; esac
  timeout -k 10 300 python3 -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline > $O/c5_$V.json 2> $O/c5_$V.err || { tail -20 $O/c5_$V.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c5_$V.json').read().strip().splitlines()[-1]); print('hb$V', d['ms_per_step'], d['roofline'].get('device_ms_per_round'))"
done
