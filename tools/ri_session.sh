# RoutingInfo compact storage / init: parity, then the default bench (warm + cold legs)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_routing_info.py tests/test_gpu_apsp.py tests/test_gpu_c_abi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ri_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/ri_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/ri_bench.txt 2>&1; rc=$?; tail -1 gpurun_out/ri_bench.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], json.dumps(d['config']['e2e'])[:1500])"; exit $rc
