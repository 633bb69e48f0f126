#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel-trace.
# Each GPU step has its own time limit; a crash/abort/timeout (rc >= 124 or a
# signal) ends the session, plain test failures (rc 1) do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
OUT=gpurun_out
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/session.log
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  LAST_RC=$rc
  echo "== $name rc=$rc" | tee -a $OUT/session.log
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 0 -a "$name" != "pytest_gpu" ]; then
    echo "stopping session after $name (rc=$rc)"; exit $rc
  fi
  return 0
}
STEPS=${STEPS:-"pytest smoke bench prof"}
for s in $STEPS; do
  case $s in
    pytest) step pytest_gpu ${PYTEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
            # the library these tests just passed with: its product-kernel fingerprints (tests/golden/validated_isa.json)
            if [ "$LAST_RC" = 0 ] && [ -z "${PYTEST_ARGS:-}" ]; then
              python spmv-vector-cache_amd/tools/record_validated.py spmv-vector-cache_amd/lib/libhipspmv.so \
                $OUT/validated_isa.json "$(grep -E '^=+ .*passed' $OUT/pytest_gpu.log | tail -1 | tr -d '=' | xargs)"
            fi ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    benchfast) step bench_fast 600 python bench.py --mode fast --no-cpu-baseline ;;
    prof) export TMPDIR=/tmp; step prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rocprof ;;
    pmc) export TMPDIR=/tmp; step pmc 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-rocprof &&
         step pmc2 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-rocprof ;;
    pmc4) step pmc4 400 bash spmv-vector-cache_amd/tools/gpurun_pmc.sh ;;
    micro) step micro 300 ./spmv-vector-cache_amd/tools/microbench ;;
    exp) HIPSPMV_EXPERIMENTAL=1 step pytest_exp 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k experimental ;;
    ablate) step ablate 600 ./spmv-vector-cache_amd/lib/vc_ablate ;;
    stamps) step stamps 300 ./spmv-vector-cache_amd/lib/vc_ablate 20 stamps ;;
    chain) step chain 120 ./spmv-vector-cache_amd/lib/chain_probe ;;
    mall) step mall88 300 ./spmv-vector-cache_amd/lib/pf_probe 88 base && step mall44 300 ./spmv-vector-cache_amd/lib/pf_probe 44 base &&
          step mall22 300 ./spmv-vector-cache_amd/lib/pf_probe 22 base ;;
    benchtime) step bench_time 900 bash -c 'time python bench.py' ;;
    mallpol) step mall_policy 300 ./spmv-vector-cache_amd/lib/pf_probe 88 mall ;;
    sweepc4c) step sweep_c4_chunks 900 python spmv-vector-cache_amd/tools/kernel_sweep.py --log2-rows 24 --log2-cols 24 --only "wgather c" --rounds 2 --reps 10 ;;
    selltests) step pytest_sell 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "sell or rmat or hub or fullsize" ;;
    sweepc4nt) step sweep_c4_nt 900 python spmv-vector-cache_amd/tools/kernel_sweep.py --log2-rows 24 --log2-cols 24 --only "=wgather,=wgather nt" --rounds 2 --reps 10 ;;
    states) step profile_states 300 python -u spmv-vector-cache_amd/tools/profile_states.py ;;
    wcsrtests) step pytest_wcsr 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "wcsr" ;;
    sweep4) HIPSPMV_EXPERIMENTAL=1 step sweep_split4 900 python spmv-vector-cache_amd/tools/kernel_sweep.py --only "split4,=vcache_split" ;;
    chainsweep) HIPSPMV_EXPERIMENTAL=1 step chain_sweep 240 python -u spmv-vector-cache_amd/tools/chain_sweep.py ;;
    wcsrshards) step wcsr_shards 900 bash -c 'for s in 0 3 7; do python -u spmv-vector-cache_amd/tools/wfast_probe.py --windows "" --shard $s || exit 1; done' &&
      HIPSPMV_WCSR_LDS=1 step wcsr_shards_lds 900 bash -c 'for s in 0 3 7; do python -u spmv-vector-cache_amd/tools/wfast_probe.py --windows "" --only-wcsr --shard $s || exit 1; done' ;;
    wcsrwin) for w in 15 17; do HIPSPMV_WCSR_LOG2W=$w step wcsr_shards_w$w 900 bash -c 'for s in 0 3 7; do python -u spmv-vector-cache_amd/tools/wfast_probe.py --windows "" --only-wcsr --shard $s || exit 1; done' || break; done &&
      step wcsr_shards_w16 900 bash -c 'for s in 0 3 7; do python -u spmv-vector-cache_amd/tools/wfast_probe.py --windows "" --only-wcsr --shard $s || exit 1; done' ;;
    wcsrcap) for c in ${CAPS:-1024 4096}; do HIPSPMV_WCSR_MAXSEG=$c step wcsr_shards_cap$c 900 bash -c 'for s in 0 3; do python -u spmv-vector-cache_amd/tools/wfast_probe.py --windows "" --only-wcsr --shard $s || exit 1; done' || break; done &&
      step wcsr_shards_nocap 900 bash -c 'for s in 0 3; do python -u spmv-vector-cache_amd/tools/wfast_probe.py --windows "" --only-wcsr --shard $s || exit 1; done' ;;
    wfast) step wfast_probe 900 python -u spmv-vector-cache_amd/tools/wfast_probe.py ;;
    wfast2) step wfast_probe_s0 600 python -u spmv-vector-cache_amd/tools/wfast_probe.py --windows 14,15,16,17 &&
            step wfast_probe_s7 600 python -u spmv-vector-cache_amd/tools/wfast_probe.py --shard 7 --windows 15,16,17,19 &&
            step wfast_probe_c4 600 python -u spmv-vector-cache_amd/tools/wfast_probe.py --c4 --windows 15,17,19 ;;
    sweepnt) step sweep_nt 900 python spmv-vector-cache_amd/tools/kernel_sweep.py --only "vcache,sell,split" ;;
    newtests) step pytest_new 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "profile or spmvbench or cache_behaviour" ;;
    sweep) step sweep 600 python spmv-vector-cache_amd/tools/kernel_sweep.py ;;
    sweepx) HIPSPMV_EXPERIMENTAL=1 step sweep_exp 900 python spmv-vector-cache_amd/tools/kernel_sweep.py ;;
    sweeprmat) step sweep_rmat 600 python spmv-vector-cache_amd/tools/kernel_sweep.py --rmat 20 ;;
    sweepwidex) HIPSPMV_EXPERIMENTAL=1 step sweep_wide_exp 600 python spmv-vector-cache_amd/tools/kernel_sweep.py --log2-rows 21 --log2-cols 24 --rounds 2 ;;
    sweepwide) step sweep_wide 600 python spmv-vector-cache_amd/tools/kernel_sweep.py --log2-rows 21 --log2-cols 24 ;;
    sweepc4) step sweep_c4 600 python spmv-vector-cache_amd/tools/kernel_sweep.py --log2-rows 24 --log2-cols 24 --only wgather --rounds 2 --reps 10 ;;
    c4) step bench_c4 900 python bench.py --workload c4 --steps 20 --warmup 5 ;;
    c5) step bench_c5 900 python bench.py --workload c5 --steps 20 --warmup 5 ;;
    c4shard) step bench_c4_shard 900 python bench.py --workload c4 --shard 0/8 --steps 50 --warmup 5 ;;
    c5shard) step bench_c5_shard 900 python bench.py --workload c5 --shard 0/8 --steps 50 --warmup 5 ;;
    c4sell) step bench_c4_sell 900 python bench.py --workload c4 --kernel sell --steps 20 --warmup 5 ;;
    c5sell) step bench_c5_sell 900 python bench.py --workload c5 --kernel sell --steps 20 --warmup 5 ;;
    c4wg) HIPSPMV_EXPERIMENTAL=1 step bench_c4_wgather 900 python bench.py --workload c4 --scale 24 --kernel wgather --mode ordered --steps 10 --warmup 3 --no-secondary ;;
    multi) step spmvbench_multi 300 ./spmv-vector-cache_amd/lib/spmvbench --dir tests/golden/matrices --confs hip,hip4 --cms 0 --reps 3 circuit204 i64k row64k ;;
  esac
done
echo "session done"
