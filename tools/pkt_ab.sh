#!/bin/bash
# Packet-stage draw-kernel shape A/B (SRT_PKT_DRAW) on C5, after the packet tests.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-pkt}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_packet.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-64x32 64x16 256x32 256x16}; do
  SRT_PKT_DRAW=$v timeout -k 10 200 python -u bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_$v.json 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step']*1e3,1), 'us/round')"
done
