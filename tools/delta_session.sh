# delta-stepping sparse sweep: parity tests, then C4 at several bucket widths
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-delta}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sssp.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in ${DELTAS:-0 0.25 0.1 0.5 1}; do
  SRT_SSSP_DELTA=$f timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-cold > $O/c4_$f.json 2>&1 || { tail -5 $O/c4_$f.json; exit 1; }
  python -c "import json; d=json.loads(open('$O/c4_$f.json').read().strip().splitlines()[-1]); c=d['config']; print('delta $f', round(d['ms_per_step'],1), c.get('plan','')[-60:], c.get('sparse_sweeps', c.get('phases_last_build')))"
done
