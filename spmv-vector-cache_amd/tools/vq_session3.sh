cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "vquad" > gpurun_out/pytest_vquad2.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_vquad2.log; exit 1; }
tail -2 gpurun_out/pytest_vquad2.log
bash spmv-vector-cache_amd/tools/vq_session2.sh
