#!/bin/bash
# one GPU session of round-5 work (edited per session): bench lines with the committed PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05lines
for c in c3 c2 c2nc c3ns c5 c4; do
  timeout -k 10 400 python3 -u bench.py --config $c --steps 10 --warmup 2 > gpurun_out/r05lines/$c.json 2> gpurun_out/r05lines/$c.err || { echo "bench $c failed"; tail -5 gpurun_out/r05lines/$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05lines/$c.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$c', d['value'], d['ms_per_step'], r.get('frac'), r.get('traffic'))"
done
