export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s1_pytest_gpu.txt 2>&1 && tail -3 gpurun_out/s1_pytest_gpu.txt &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s1_smoke.txt 2>&1 && tail -2 gpurun_out/s1_smoke.txt &&
timeout -k 10 400 python -u bench.py > gpurun_out/s1_bench.txt 2>&1; tail -1 gpurun_out/s1_bench.txt
