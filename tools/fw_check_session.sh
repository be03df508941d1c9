export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fw_pair.py tests/test_gpu_apsp.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fin_pytest.txt 2>&1 && tail -2 gpurun_out/fin_pytest.txt &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/fin_c3.txt 2>&1 && tail -1 gpurun_out/fin_c3.txt | cut -c 380-800
