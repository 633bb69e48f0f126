# C5 per-shard block (cost partition) at wcsr windows 2^18 and 2^19 (probe env)
cd $GRAFT_REPO_ROOT
for w in 20 21 22; do
  HIPSPMV_WCSR_LOG2W=$w timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-strong --no-rocprof > gpurun_out/bench_c5_w$w.log 2>&1 || { echo c5 w$w failed; tail -20 gpurun_out/bench_c5_w$w.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_c5_w$w.log') if l.startswith('{')][-1]); c=d['c5_shards']
print('w$w', c.get('error'), c.get('max_over_min'), c.get('slowest_us'), c.get('min_roofline_frac'))
for s in c.get('shards', []): print(s['shard'], s['nnz'], s['kernel'], s.get('kernel_us'), s.get('roofline_frac'), s.get('segments'))
"
done
