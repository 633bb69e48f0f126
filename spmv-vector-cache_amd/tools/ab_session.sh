# A/B of the C3 FAST kernels in one box: vcache_split (k_vcache, three parts)
# clamped (xlane 3) vs masked (xlane 4) entry loads, and k_vquad; two rounds
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for k in split3 split3m vq18; do
    case $k in
      split3) extra="--kernel vcache_split --vcache-xlane 3" ;;
      split3m) extra="--kernel vcache_split --vcache-xlane 4" ;;
      vq18) extra="--kernel vcache_split4 --vquad-variant 18" ;;
    esac
    timeout -k 10 240 python bench.py $extra --steps 200 --warmup 20 --no-cpu-baseline --no-secondary --no-strong --no-rocprof --no-c5-shards > gpurun_out/ab_${k}_$r.log 2>&1 || { echo bench $k failed; tail -20 gpurun_out/ab_${k}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_${k}_$r.log') if l.startswith('{')][-1]); r=d['roofline']; print('$k round $r', r['kernel_us'], r['frac'], d['ms_per_step'])"
  done
done
