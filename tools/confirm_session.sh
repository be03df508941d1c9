# round-end rehearsal on one GPU: the whole -m gpu suite, smoke(), the default
# bench line (C3 with its CPU baseline).  usage: bash tools/confirm_session.sh [tag]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-confirm}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
tail -1 $O/c3.json | cut -c1-300
