#!/bin/bash
# round-6 session 49: bench lines with the level roofline second peak / write floor
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6rl
for C in c3 c3ns; do
timeout -k 10 300 python3 -u bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-cold > gpurun_out/r6rl/$C.json 2> gpurun_out/r6rl/$C.err || { tail -20 gpurun_out/r6rl/$C.err; exit 1; }
python3 -c "import json; d=json.loads(open(\"gpurun_out/r6rl/$C.json\").read().strip().splitlines()[-1]); r=d[\"roofline\"]; print(\"$C\", d[\"ms_per_step\"], r[\"frac\"], r[\"second_peak\"][\"frac\"], r[\"write_floor\"][\"frac_of_hbm\"])"
done
