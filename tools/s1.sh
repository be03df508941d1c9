set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_packet.py tests/test_golden.py tests/test_packet_events.py -m gpu > gpurun_out/s1/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/s1/tests.log; exit 1; }
tail -3 gpurun_out/s1/tests.log
bash tools/profile_round.sh r06c5 --config c5 --steps 50 --warmup 5 || exit 1
