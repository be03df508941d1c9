# event push: parity tests, then a C5 kernel trace (per-kernel averages)
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-ev}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_packet_events.py tests/test_gpu_packet.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 $R/bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
timeout -k 10 200 python3 $R/bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5.json 2>&1
