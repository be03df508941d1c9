#!/bin/bash
# Dense multi-GPU critical-path emulation on one GPU (bench.py --emulate-ranks)
# plus the sharded-path parity tests.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-emu}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_apsp.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/c3.json 2>&1 || exit 1
python -c "import json; d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]); print('c3 1gpu', round(d['ms_per_step'],2), round(d['roofline']['frac'],4))"
for n in 2 4 8; do
  timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --emulate-ranks $n > $O/emu$n.json 2>&1 || exit 1
  tail -1 $O/emu$n.json
  SRT_FW_NO_SMALL_CHAIN=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --emulate-ranks $n > $O/emu${n}_big.json 2>&1 || exit 1
  tail -1 $O/emu${n}_big.json
done
