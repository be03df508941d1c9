# chain-kernel change: parity tests (1 GPU + gloo ranks), the isolated probe, emulated 8/4 ranks
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-q16}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fw_pair.py tests/test_gpu_apsp.py tests/test_gpu_dist.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/chain_probe.sh || exit 1
for n in 8 4; do
  for g in 1 2; do
    SRT_FW_SYM_GROUP=$g timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cold --no-e2e --emulate-ranks $n > $O/emu${n}_g$g.json 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$O/emu${n}_g$g.json').read().strip().splitlines()[-1]); print('ranks $n g $g', round(d['ms_per_step'],3), d['rest_launches_per_step'], round(d['rest_ms_per_step'],2), d['tail_ms_last'])"
  done
done
