# squaring phase 1: parity tests, then emulated 8/4-rank C3 (g = 1, 2) and a trace of 8 ranks g = 2
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-p1sq}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fw_pair.py -k "phase1" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dist.py -k "undirected" > $O/tests_dist.log 2>&1 || { tail -40 $O/tests_dist.log; exit 1; }
tail -2 $O/tests_dist.log
for n in 8 4; do
  for g in 1 2; do
    SRT_FW_SYM_GROUP=$g timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cold --no-e2e --emulate-ranks $n > $O/emu${n}_g$g.json 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$O/emu${n}_g$g.json').read().strip().splitlines()[-1]); print('ranks $n g $g', round(d['ms_per_step'],3), d['rest_launches_per_step'], round(d['rest_ms_per_step'],2), d['tail_ms_last'])"
  done
done
SRT_FW_SYM_GROUP=2 EMU_TAG=g2sq bash tools/emu_trace.sh 8
