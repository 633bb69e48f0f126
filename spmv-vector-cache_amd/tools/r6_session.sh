#!/bin/bash
# Round-6 GPU session steps (each with its own time limit; a crash/abort/timeout ends the session).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/session.log
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/session.log
  tail -4 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 1 ]; then echo "stopping session after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
for s in ${STEPS:-streams}; do
  case $s in
    streams) step pytest_streams 400 $PYT -m gpu tests/test_gpu_streams.py -s ;;
    scratch) step pytest_scratch 600 $PYT -m gpu tests/test_gpu_parity.py -k "split or sell or wcsr or graph or concurrent" ;;
    multi) step pytest_multi 600 $PYT -m gpu tests/test_gpu_multi.py ;;
    gaps) step gaps 300 rocprofv3 --kernel-trace -d $OUT/gaps -o run --output-format csv -- python3 spmv-vector-cache_amd/tools/launch_gaps.py --launches 40 &&
          step gaps_summary 60 python3 spmv-vector-cache_amd/tools/launch_gaps_csv.py $OUT/gaps 40 ;;
    vflow) step pytest_vflow 300 $PYT -m gpu tests/test_gpu_parity.py -k "vcache_flow or vflow" ;;
    vfprof) step vf_prof 300 python -u spmv-vector-cache_amd/tools/vf_prof.py ${VFPROF_ARGS:-} ;;
    vfab) step vf_ab 300 python -u spmv-vector-cache_amd/tools/vf_ab.py ${VFAB_ARGS:-} ;;
    pmcord) KERNELS=vcache WORKLOAD=c3 step pmc_ordered 600 bash spmv-vector-cache_amd/tools/gpurun_pmc.sh &&
            step pmc_ordered_summary 60 python3 spmv-vector-cache_amd/tools/pmc_summary.py $OUT/pmc_c3_vcache_summary.csv "k_vcache<double, 1," $OUT/pmc_c3_vcache_*/*counter_collection.csv ;;
    destroy) HIPSPMV_SYNC_RELEASE=1 step destroy_sync 300 python -u spmv-vector-cache_amd/tools/destroy_probe.py &&
             step destroy_deferred 300 python -u spmv-vector-cache_amd/tools/destroy_probe.py &&
             HIPSPMV_SYNC_RELEASE=1 step destroy_sync_trace 300 rocprofv3 --kernel-trace -d $OUT/destroy_sync -o run --output-format csv -- python3 spmv-vector-cache_amd/tools/destroy_probe.py &&
             step destroy_deferred_trace 300 rocprofv3 --kernel-trace -d $OUT/destroy_deferred -o run --output-format csv -- python3 spmv-vector-cache_amd/tools/destroy_probe.py ;;
    wgstests) step pytest_wgs 600 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_fullsize.py -k "wgather or c4_shard" ;;
    wgsab) step wgs_ab 400 python -u spmv-vector-cache_amd/tools/wgs_ab.py ${WGSAB_ARGS:-} ;;
    wgsnt) step wgs_nt 600 python -u spmv-vector-cache_amd/tools/wgs_ab.py --kernels wgather_split --nt ${WGS_NT:-0,12,20,28,40} --shards ${WGS_SHARDS:-0} ;;
    streams2) step pytest_streams2 400 $PYT -m gpu tests/test_gpu_streams.py tests/test_gpu_parity.py -k "wgather_split" ;;
    c5xcd) step c5_xcd 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set xcd --shards 0,3,7 ;;
    c5xcd19) HIPSPMV_WCSR_LOG2W=19 step c5_xcd_w19 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set xcd --shards 0,3,7 ;;
    c5xcd18) HIPSPMV_WCSR_LOG2W=18 step c5_xcd_w18 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set xcd --shards 0,3,7 ;;
    pmcc4s) KERNELS="wgather_split wgather" WORKLOAD=c4s7 step pmc_c4s7 900 bash spmv-vector-cache_amd/tools/gpurun_pmc.sh &&
            step pmc_c4s7_split_summary 60 python3 spmv-vector-cache_amd/tools/pmc_summary.py $OUT/pmc_c4s7_wgather_split_summary.csv "k_wgather_split<double," $OUT/pmc_c4s7_wgather_split_*/*counter_collection.csv &&
            step pmc_c4s7_wg_summary 60 python3 spmv-vector-cache_amd/tools/pmc_summary.py $OUT/pmc_c4s7_wgather_summary.csv "k_wgather<double," $OUT/pmc_c4s7_wgather_[0-9]*/*counter_collection.csv ;;
    c5wg) step c5_wg 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set wg --shards 0,3,7 ;;
    whole) step pytest_whole 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "whole or c4_shard or random_ragged" ;;
    wgsmap) step wgs_map 600 python -u spmv-vector-cache_amd/tools/wgs_ab.py --kernels "wgather,wgather_split,wgather_split#alt" --rounds 4 ;;
    hottests) HIPSPMV_EXPERIMENTAL=1 HIPSPMV_WCSR_HOT=16384 step pytest_hot 600 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_multi.py -k "wcsr" &&
              HIPSPMV_EXPERIMENTAL=1 HIPSPMV_WCSR_HOT=8192 step pytest_hot8k 600 $PYT -m gpu tests/test_gpu_parity.py -k "wcsr" ;;
    hotab) step c5_hot_off 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set one --shards 0,3,7 &&
           HIPSPMV_EXPERIMENTAL=1 HIPSPMV_WCSR_HOT=16384 step c5_hot_16k 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set one --shards 0,3,7 &&
           HIPSPMV_EXPERIMENTAL=1 HIPSPMV_WCSR_HOT=8192 step c5_hot_8k 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set one --shards 0,3,7 ;;
    hotab2) step c5_hot_off 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set one --shards 0,3,7 &&
            HIPSPMV_EXPERIMENTAL=1 HIPSPMV_WCSR_HOT=8192 step c5_hot_8k 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set one --shards 0,3,7 ;;
    ldsab) step c5_lds_off 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set one --shards 0,3,7 &&
           HIPSPMV_WCSR_LDS=1 step c5_lds_on 600 python -u spmv-vector-cache_amd/tools/c5_ab.py --set one --shards 0,3,7 ;;
    wgs4) HIPSPMV_WGS_MAXROWS=16777216 step wgs_ab4 600 python -u spmv-vector-cache_amd/tools/wgs_ab.py --parts 4 --shards 0 &&
          HIPSPMV_WGS_MAXROWS=16777216 step wgs_ab2 600 python -u spmv-vector-cache_amd/tools/wgs_ab.py --parts 2 --shards 0 --rounds 2 --launches 20 ;;
    graph) step pytest_graph 300 $PYT -m gpu tests/test_gpu_parity.py -k "graph_capture" ;;
    dmawait) step dmawait 300 ./spmv-vector-cache_amd/lib/vc_ablate 20 dmawait ;;
    pytest) step pytest_gpu 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench) step bench 600 python bench.py ;;
    bench20) step bench20 600 python bench.py --steps 20 --warmup 5 ;;
  esac
done
echo "session done"
