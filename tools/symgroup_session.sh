# grouped symmetric sharded schedule: the gloo multi-rank parity tests, then
# emulated C3 at 4 / 8 ranks for SRT_FW_SYM_GROUP = 1 / 2 / 4
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-symgroup}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dist.py -k "undirected" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for n in 4 8; do
  for g in 1 2 4; do
    SRT_FW_SYM_GROUP=$g timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cold --emulate-ranks $n > $O/emu${n}_g$g.json 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$O/emu${n}_g$g.json').read().strip().splitlines()[-1]); print('ranks $n g $g', round(d['ms_per_step'],3), d['rest_launches_per_step'], round(d['rest_ms_per_step'],2), d['tail_ms_last'])"
  done
done
