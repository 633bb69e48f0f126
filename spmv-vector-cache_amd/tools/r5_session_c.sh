#!/bin/bash
# round 5 session c: the GPU suite on the banked layouts + xlane 5, record the validated machine code,
# then the driver's bench command
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05/pytest_gpu_c.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r05/pytest_gpu_c.log; exit 1; }
summary=$(tail -1 gpurun_out/r05/pytest_gpu_c.log | tr -d '=')
echo "$summary"
python3 spmv-vector-cache_amd/tools/record_validated.py spmv-vector-cache_amd/lib/libhipspmv.so \
  gpurun_out/r05/validated_isa.json "pytest -m gpu:$summary (profiles/r05/logs/pytest_gpu_c.log)" || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05/bench_c.log 2> gpurun_out/r05/bench_c.err || { echo "bench rc=$?"; tail -20 gpurun_out/r05/bench_c.err; exit 1; }
tail -c 3000 gpurun_out/r05/bench_c.log
