# level fold: parity (GPU tests touching the dense loss pass), then the C3
# bench with the level fold and with the scan fold (SRT_LOSS_LEVEL=0)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_apsp.py tests/test_gpu_configs.py tests/test_gpu_dist.py tests/test_gpu_fw_pair.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lv_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/lv_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/lv_bench.txt 2>&1 && tail -1 gpurun_out/lv_bench.txt | cut -c1-1500 &&
SRT_LOSS_LEVEL=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/lv_bench_scan.txt 2>&1 && tail -1 gpurun_out/lv_bench_scan.txt | cut -c1-900
