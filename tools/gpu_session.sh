#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s57
for v in 0 32 40 48 0 40; do
SRT_FR_SECOND=$v timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-cold > gpurun_out/s57/v$v.json 2> gpurun_out/s57/v$v.err || { echo "bench $v failed"; tail -5 gpurun_out/s57/v$v.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s57/v$v.json').read().strip().splitlines()[-1]); print('second $v', d['ms_per_step'], d['roofline'].get('launches_per_step'), d['roofline']['schedule'].get('blocks'))"
done
