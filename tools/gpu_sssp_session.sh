#!/bin/bash
# GPU session: full GPU test suite, then the sparse (C4) build at growing
# in-use counts, then the default C3 line.  Every GPU step has its own limit
# and the chain stops at the first failure.
export TMPDIR=/tmp
O=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-sssp}
mkdir -p $O
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -5 $O/pytest_gpu.txt; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --config c4 --in-use 4096 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4_4k.json 2> $O/c4_4k.err
rc=$?; tail -1 $O/c4_4k.json; echo "c4_4k rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > $O/c4_full.json 2> $O/c4_full.err
rc=$?; tail -1 $O/c4_full.json; echo "c4_full rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err
rc=$?; tail -1 $O/c3.json; echo "c3 rc=$rc"
