# rocprof kernel split (segment pass / reduce) of C5 shards 0 and 7 of 8 (cost partition)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for sh in 0 7; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$sh -o run --output-format csv -- python3 bench.py --workload c5 --shard $sh/8 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-strong --no-rocprof --no-c5-shards > gpurun_out/prof_c5_$sh.log 2>&1 || { echo shard $sh failed; tail -5 gpurun_out/prof_c5_$sh.log; exit 1; }
  echo "shard $sh"; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_c5_$sh/run_kernel_stats.csv')): print('  ', r['Name'][:60], r['Calls'], r['AverageNs'])
"
done
