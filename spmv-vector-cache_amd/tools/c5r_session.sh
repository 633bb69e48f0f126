# wcsr lane reduce: parity (wcsr tests, full-size C5 u64 / sampled), then the C5 shard block and the split
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "wcsr or c5" > gpurun_out/pytest_c5r.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_c5r.log; exit 1; }
tail -n 1 gpurun_out/pytest_c5r.log
timeout -k 10 600 python bench.py --no-cpu-baseline --no-secondary --no-rocprof --no-strong --steps 20 --warmup 5 > gpurun_out/bench_c5r.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_c5r.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_c5r.log') if l.startswith('{')][-1])
c=d['c5_shards']; print('C5', c.get('max_over_min'), c.get('slowest_us'), c.get('min_roofline_frac'))
for s in c.get('shards', []): print(s['shard'], s['nnz'], s['kernel'], s.get('kernel_us'), s.get('roofline_frac'), s.get('parity'))
"
bash spmv-vector-cache_amd/tools/c5_prof_session.sh
