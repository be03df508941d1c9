# Round-3 final evidence besides the C3 profile (tools/profile_round.sh r03f_c3):
# the other configs' bench lines, the C4 round profile (trace + FETCH/WRITE),
# and the emulated 2/4/8-rank C3 builds (plus the 8-rank all-gather model at
# 400 GB/s for sensitivity).  usage: bash tools/r03f_profiles.sh [part]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out/r03f
if [ "${1:-all}" != "emu" ]; then
  for c in c1 c2 c2nc c5; do
    timeout -k 10 400 python -u bench.py --config $c > gpurun_out/r03f/$c.json 2> gpurun_out/r03f/$c.err || { tail -5 gpurun_out/r03f/$c.err; exit 1; }
    tail -1 gpurun_out/r03f/$c.json | cut -c1-200
  done
  bash tools/profile_round.sh r03f_c4 --config c4 || exit 1
fi
if [ "${1:-all}" != "cfg" ]; then
  for n in 2 4 8; do
    timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold --no-e2e --emulate-ranks $n > gpurun_out/r03f/emu$n.json 2>&1 || exit 1
    grep '^{' gpurun_out/r03f/emu$n.json | tail -1 | cut -c1-160
  done
  SRT_FW_EMU_AG_GBPS=400 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold --no-e2e --emulate-ranks 8 > gpurun_out/r03f/emu8_400.json 2>&1 || exit 1
  grep '^{' gpurun_out/r03f/emu8_400.json | tail -1 | cut -c1-160
fi
