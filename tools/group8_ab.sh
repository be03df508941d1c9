export TMPDIR=/tmp; mkdir -p gpurun_out
SRT_FW_GROUP=8 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/grp_c3_g8.txt 2>&1 && tail -1 gpurun_out/grp_c3_g8.txt | cut -c 300-1000 &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/grp_c3_g4b.txt 2>&1 && tail -1 gpurun_out/grp_c3_g4b.txt | cut -c 300-1000 &&
SRT_FW_PAIR=1 SRT_FW_GROUP=8 timeout -k 10 200 python -u -m pytest tests/test_gpu_fw_pair.py -x -q --timeout 120 --timeout-method thread -k "1000 or 1500" > gpurun_out/grp8_pytest.txt 2>&1; tail -2 gpurun_out/grp8_pytest.txt
