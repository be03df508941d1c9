export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for v in libsrt libsrt_noremap libsrt libsrt_noremap; do
  SRT_LIB=$PWD/shadow_amd/$v.so timeout -k 10 200 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab.json 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],1))"
done
