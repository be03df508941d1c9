#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s30
timeout -k 10 900 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_level.py tests/test_gpu_configs.py tests/test_gpu_apsp.py tests/test_gpu_routing_info.py > gpurun_out/s30/tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/s30/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/s30/tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s30/t -o run --output-format csv -- python3 $R/bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-cold > $R/gpurun_out/s30/t.log 2>&1 || { echo "trace failed"; exit 1; }
python3 - $R/gpurun_out/s30/t <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r['Name'][:80].ljust(80), r['Calls'].rjust(5), '%.3f ms avg' % (float(r['AverageNs'])/1e6))
PY
cd $R
SRT_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/s30/c3.json 2> gpurun_out/s30/c3.err || { echo "bench failed"; tail -5 gpurun_out/s30/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s30/c3.json').read().strip().splitlines()[-1]); e=d['config']['e2e']; print(d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'), e['ms'], e['routing_info']['ms'])"
grep -E "e2e:|create: level" gpurun_out/s30/c3.err | tail -9
