#!/bin/bash
# round-6 session 33: same-box A/B of the source-offset prefetch (libsrt.so) against without (libsrt_alt.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6soff
mkdir -p $O
export TMPDIR=/tmp
for V in soff alt soff2 alt2; do
  case $V in alt*) export SRT_LIB=$GRAFT_REPO_ROOT/shadow_amd/libsrt_alt.so;; *) unset SRT_LIB;; esac
  for C in c3 c2; do
  timeout -k 10 300 python3 -u bench.py --config $C --steps 10 --warmup 3 --no-cold --no-cpu-baseline --no-e2e > $O/${C}_$V.json 2> $O/${C}_$V.err || { tail -20 $O/${C}_$V.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/${C}_$V.json').read().strip().splitlines()[-1]); c=d['config']; print('$C $V', d['ms_per_step'], c['phases_last_build']['dominant_ms'])"
  done
done
