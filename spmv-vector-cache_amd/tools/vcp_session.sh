# split-geometry ring-shape probes on C3 FAST (HIPSPMV_VC_PROBE), interleaved, two rounds
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for p in 0 1 2 3; do
    HIPSPMV_VC_PROBE=$p timeout -k 10 240 python bench.py --kernel vcache_split --steps 200 --warmup 20 --no-cpu-baseline --no-secondary --no-strong --no-rocprof --no-c5-shards > gpurun_out/vcp_${p}_$r.log 2>&1 || { echo probe $p failed; tail -20 gpurun_out/vcp_${p}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/vcp_${p}_$r.log') if l.startswith('{')][-1]); r=d['roofline']; print('probe $p round $r', r['kernel_us'], r['frac'], d['parity'])"
  done
done
