#!/bin/bash
# round 5 session a: k_vquad variants 21-26 parity, then the steady-state A/B sweep
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "vquad_variants" > gpurun_out/r05/pytest_vquad_a.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05/pytest_vquad_a.log; exit 1; }
tail -2 gpurun_out/r05/pytest_vquad_a.log
timeout -k 10 300 python -u spmv-vector-cache_amd/tools/ab_sweep.py --set vquad --rounds 3 > gpurun_out/r05/ab_vquad_a.log 2>&1 || { echo "sweep rc=$?"; tail -20 gpurun_out/r05/ab_vquad_a.log; exit 1; }
cat gpurun_out/r05/ab_vquad_a.log
