# chain-kernel latency probe under a kernel trace (see tools/chain_probe.hip)
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/chain_probe
mkdir -p $O
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- $R/tools/chain_probe.bin > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
tail -2 $O/run.log
