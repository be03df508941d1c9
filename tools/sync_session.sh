# emulated 8/4-rank C3 at g = 2: event hand-offs vs stream memory operations; 2 ranks g = 1 / 2
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-sync}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dist.py -k "s2 or s4 or s3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
SRT_FW_SYNC=value timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dist.py -k "s2 or s4 or s3" >> $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep passed $O/tests.log
run() { timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold --no-e2e --emulate-ranks $1 > $O/$2.json 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$O/$2.json').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],3), round(d['rest_ms_per_step'],2), d['tail_ms_last'])"; }
for n in 8 4; do
  SRT_FW_SYM_GROUP=2 run $n emu${n}_g2_event
  SRT_FW_SYM_GROUP=2 SRT_FW_SYNC=value run $n emu${n}_g2_value
done
SRT_FW_SYM_GROUP=1 run 2 emu2_g1
SRT_FW_SYM_GROUP=2 run 2 emu2_g2
SRT_FW_SYM_GROUP=2 SRT_FW_SYNC=value run 2 emu2_g2_value
