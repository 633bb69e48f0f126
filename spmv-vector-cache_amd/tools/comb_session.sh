# owner-combine check: the vcache-family parity tests, then the C3 FAST A/B
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "vcache_split_entry or vquad_variants or c3" > gpurun_out/pytest_comb.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_comb.log; exit 1; }
tail -2 gpurun_out/pytest_comb.log
bash spmv-vector-cache_amd/tools/ab_session.sh
