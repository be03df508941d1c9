#!/bin/bash
# FW staging A/B: parity tests on the default (glds) kernel, then C2/C3 bench
# lines for both staging variants.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-fwstage}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_apsp.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for st in glds reg; do
  for cf in c2 c3; do
    SRT_FW_STAGE=$st timeout -k 10 200 python -u bench.py --config $cf --steps 3 --warmup 1 --no-cpu-baseline > $O/${cf}_$st.json 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$O/${cf}_$st.json').read().strip().splitlines()[-1]); print('$cf $st', round(d['ms_per_step'],2), round(d['roofline']['frac'],4), d['roofline']['avg_launch_ms'])"
  done
done
