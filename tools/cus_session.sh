# emulated 8-rank C3 (g = 2) with c CUs kept free of the rest launch for the chain
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-cus}
mkdir -p $O
cd $R
for c in 0 8 16 32 64; do
  SRT_FW_CHAIN_CUS=$c SRT_FW_CHAIN_CU_STRIDE=1 SRT_FW_SYM_GROUP=2 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cold --no-e2e --emulate-ranks 8 > $O/emu8_c$c.json 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$O/emu8_c$c.json').read().strip().splitlines()[-1]); print('cus $c', round(d['ms_per_step'],3), round(d['rest_ms_per_step'],2), d['tail_ms_last'])"
done
