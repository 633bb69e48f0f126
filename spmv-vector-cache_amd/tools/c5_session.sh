# C5 per-shard block of bench.py under both partitions (round 4)
cd $GRAFT_REPO_ROOT
for part in cost; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-strong --no-rocprof --c5-partition $part > gpurun_out/bench_c5_$part.log 2>&1 || { echo c5 $part failed; tail -20 gpurun_out/bench_c5_$part.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_c5_$part.log') if l.startswith('{')][-1]); c=d['c5_shards']
print('$part', c.get('error'), c.get('max_over_min'), c.get('slowest_us'), c.get('min_roofline_frac'))
for s in c.get('shards', []): print(s['shard'], s['rows'], s['nnz'], s['kernel'], s.get('kernel_us'), s.get('roofline_frac'), s.get('segments'), s.get('parity'), s.get('gen_s'), s.get('setup_s'))
"
done
