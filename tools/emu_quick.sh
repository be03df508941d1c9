# emulated N-rank C3 builds (bench.py --emulate-ranks), C2 one GPU, no tests
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-emuq}
mkdir -p $O
cd $R
timeout -k 10 200 python -u bench.py --config c2 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $O/c2.json 2>&1 || exit 1
python -c "import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); print('c2 1gpu', round(d['ms_per_step'],3), d['config']['phases_last_build'])"
for n in 2 4 8; do
  timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --emulate-ranks $n > $O/emu$n.json 2>&1 || exit 1
  tail -1 $O/emu$n.json | cut -c1-200
done
