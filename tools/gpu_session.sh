#!/bin/bash
# one GPU session of round-5 work (edited per session)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s18
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_apsp.py tests/test_gpu_routing_info.py > gpurun_out/s18/tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/s18/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/s18/tests.log
SRT_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/s18/e2e.json 2> gpurun_out/s18/e2e.err || { echo "e2e failed"; tail -5 gpurun_out/s18/e2e.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s18/e2e.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'), d['config']['e2e']['ms'], d['config']['e2e']['routing_info']['ms'])"
grep -E "e2e:|create: level|loss pieces|fetch8: pieces" gpurun_out/s18/e2e.err | tail -12
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s18/c3 -o run --output-format csv -- python3 $R/bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-cold > $R/gpurun_out/s18/c3.log 2>&1 || { echo "trace failed"; exit 1; }
python3 - $R/gpurun_out/s18/c3 <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:5]:
    print(r['Name'][:70].ljust(70), r['Calls'].rjust(5), '%.3f ms avg' % (float(r['AverageNs'])/1e6))
PY
