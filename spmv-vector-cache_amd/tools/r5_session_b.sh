#!/bin/bash
# round 5 session b: the GPU suite on the banked split layout, the A/B, and PMC passes of the product kernel
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05/pytest_gpu_b.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r05/pytest_gpu_b.log; exit 1; }
tail -3 gpurun_out/r05/pytest_gpu_b.log
timeout -k 10 200 python -u spmv-vector-cache_amd/tools/ab_sweep.py --set bank --rounds 5 > gpurun_out/r05/ab_bank_b.log 2>&1 || { echo "sweep rc=$?"; tail -20 gpurun_out/r05/ab_bank_b.log; exit 1; }
cat gpurun_out/r05/ab_bank_b.log
PASS_TIMEOUT=90 bash spmv-vector-cache_amd/tools/gpurun_pmc.sh > gpurun_out/r05/pmc_b.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/r05/pmc_b.log; exit 1; }
python3 spmv-vector-cache_amd/tools/pmc_summary.py gpurun_out/r05/pmc_c3_split_b.csv "k_vcache<double, 3" $(find gpurun_out/pmc_c3_vcache_split_* -name "*counter_collection.csv" | sort) > gpurun_out/r05/pmc_b_summary.txt 2>&1; tail -40 gpurun_out/r05/pmc_b_summary.txt
