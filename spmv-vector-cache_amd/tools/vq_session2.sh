cd $GRAFT_REPO_ROOT
for v in 0 1 3 5 17 18 19 8; do
  timeout -k 10 240 python bench.py --kernel vcache_split4 --vquad-variant $v --steps 100 --warmup 10 --no-cpu-baseline --no-secondary --no-strong --no-rocprof --no-c5-shards > gpurun_out/bench_vq$v.log 2>&1 || { echo bench $v failed; tail -20 gpurun_out/bench_vq$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_vq$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('variant $v', r['kernel_us'], r['frac'], r['kernel_us_per_launch']['median'])"
done
