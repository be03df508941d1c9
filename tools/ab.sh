#!/bin/bash
# Generic knob A/B on one GPU box: optional parity tests, then the same bench
# command once per knob set, printing ms/step and the plan for each.
# Measurement tool; replaces the one-off A/B scripts of rounds 1-2.
#   usage: [TESTS="tests/test_gpu_sssp.py"] bash tools/ab.sh OUT "BENCH ARGS" "KNOBS A" "KNOBS B" ...
#   e.g.   bash tools/ab.sh c4ab "--config c4 --steps 1 --warmup 0" "" "SRT_SSSP_SPLIT=1"
#          (a knob set is a space-separated list of VAR=value, "" = defaults;
#           every set runs twice, interleaved, to expose box noise)
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-ab}
BARGS=$2
shift 2
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
  rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  i=0
  for knobs in "$@"; do
    i=$((i + 1))
    env $knobs timeout -k 10 400 python -u bench.py $BARGS --no-cpu-baseline > $O/run${i}_$rep.json 2> $O/run${i}_$rep.err || { tail -5 $O/run${i}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/run${i}_$rep.json').read().strip().splitlines()[-1]); cf=d['config'] if isinstance(d.get('config'),dict) else {}; ph=cf.get('phases_last_build') or {}; print('[$knobs]', round(d['ms_per_step'],2), 'loss', round(ph.get('exact_loss_pass_ms',d.get('tail_ms_last',0)),2), 'rest', round(ph.get('dominant_ms',d.get('rest_ms_per_step',0)),2), cf.get('plan','')[:60])"
  done
done
