export TMPDIR=/tmp; mkdir -p gpurun_out/cl1
timeout -k 10 500 python -u -m pytest tests/test_gpu_sssp.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cl1/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/cl1/pytest.txt; [ $rc -eq 0 ] || exit $rc
CFGS="cl keys SRT_SSSP_CL=0" bash tools/c4_sweeps.sh cl1/sw 8192 || exit 1
bash tools/ab.sh cl1/full "--config c4 --steps 1 --warmup 0" "" "SRT_SSSP_CL=0"
