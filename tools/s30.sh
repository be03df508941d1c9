#!/bin/bash
# round-6 session 30: C4 sweep chunk order A/B (SRT_FR_VMAJOR: 0 block-major, 1 latency sweeps, 2 loss sweeps, 3 both)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6vm
mkdir -p $O
export TMPDIR=/tmp
for V in 0 2 3 1; do
  export SRT_FR_VMAJOR=$V
  timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --no-cold --no-cpu-baseline --no-e2e > $O/c4_$V.json 2> $O/c4_$V.err || { echo "bench $V failed"; tail -20 $O/c4_$V.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$V.json').read().strip().splitlines()[-1]); print('vm$V', d['ms_per_step'], d['config'].get('phases_last_build'))"
done
