# Round-3 evidence: the C3 round profile (bench line with CPU baseline, kernel
# trace, FETCH/WRITE and SQ PMC passes), then the other configs' bench lines.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
SQPMC=1 bash tools/profile_round.sh r03c3 || exit 1
for c in c2 c2nc c1 c5; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/r03_$c.json 2> gpurun_out/r03_$c.err || { tail -5 gpurun_out/r03_$c.err; exit 1; }
  tail -1 gpurun_out/r03_$c.json | cut -c1-300
done
bash tools/profile_round.sh r03c2 --config c2 || exit 1
timeout -k 10 600 python -u bench.py --config c4 > gpurun_out/r03_c4.json 2> gpurun_out/r03_c4.err || { tail -5 gpurun_out/r03_c4.err; exit 1; }
tail -1 gpurun_out/r03_c4.json | cut -c1-300
