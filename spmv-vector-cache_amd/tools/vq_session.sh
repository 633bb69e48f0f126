cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "vquad or split4" > gpurun_out/pytest_vquad.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_vquad.log; exit 1; }
tail -3 gpurun_out/pytest_vquad.log
for v in 0 1 2 3 4; do
  timeout -k 10 240 python bench.py --kernel vcache_split4 --vquad-variant $v --steps 100 --warmup 10 --no-cpu-baseline --no-secondary --no-strong --no-rocprof --no-c5-shards > gpurun_out/bench_vq$v.log 2>&1 || { echo bench $v failed; tail -20 gpurun_out/bench_vq$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_vq$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('variant $v', r['kernel_us'], r['frac'], r['kernel_us_per_launch']['median'], d['parity'])"
done
timeout -k 10 240 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-secondary --no-strong --no-rocprof --no-c5-shards > gpurun_out/bench_split3.log 2>&1 && python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bench_split3.log') if l.startswith('{')][-1]); r=d['roofline']; print('split3', r['kernel_us'], r['frac'], r['kernel_us_per_launch']['median'])"
