# round-4 check: wcsr / wgather parity, then the bench without the CPU legs (C3, C4 strong, C5 shards)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "wcsr or wgather or c5" > gpurun_out/pytest_r4.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_r4.log; exit 1; }
tail -n 1 gpurun_out/pytest_r4.log
timeout -k 10 700 python bench.py --no-cpu-baseline --no-secondary --no-rocprof > gpurun_out/bench_r4.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_r4.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_r4.log') if l.startswith('{')][-1])
st=d['strong']; print('C3', d['roofline']['frac'], d['roofline']['kernel_us']); print('C4', {k:st[k] for k in ('kernel','roofline_frac_rank0','setup_s','setup_ns_lib','setup_phases_ns','ms_per_step')})
c=d['c5_shards']; print('C5', c.get('max_over_min'), c.get('slowest_us'), c.get('min_roofline_frac'))
for s in c.get('shards', []): print(s['shard'], s['nnz'], s['kernel'], s.get('kernel_us'), s.get('roofline_frac'), s.get('segments'), s.get('parity'))
"
timeout -k 10 300 python spmv-vector-cache_amd/tools/kernel_sweep.py --log2-rows 24 --log2-cols 24 --only "=wgather" --rounds 2 --reps 10 > gpurun_out/sweep_c4_masked.log 2>&1 || { echo sweep c4 failed; tail -5 gpurun_out/sweep_c4_masked.log; exit 1; }
tail -n 1 gpurun_out/sweep_c4_masked.log
timeout -k 10 300 python spmv-vector-cache_amd/tools/kernel_sweep.py --only "=wgather,=sell" --rounds 2 --reps 20 > gpurun_out/sweep_c3_wgather.log 2>&1 || { echo sweep c3 failed; tail -5 gpurun_out/sweep_c3_wgather.log; exit 1; }
tail -n 3 gpurun_out/sweep_c3_wgather.log
