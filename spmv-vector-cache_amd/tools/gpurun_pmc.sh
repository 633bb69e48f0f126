# rocprofv3 --pmc passes (one counter group per run) of one kernel on one
# workload: KERNELS / WORKLOAD env (default vcache_split on C3)
export TMPDIR=/tmp
P0="FETCH_SIZE"
P5="WRITE_SIZE"
P1="TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCP_UTCL1_SERIALIZATION_STALL TCP_UTCL1_STALL_INFLIGHT_MAX TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_MULTI_MISS TCP_TCR_TCP_STALL_CYCLES TD_TD_BUSY TD_TC_STALL SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P3="TCC_HIT TCC_MISS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM"
P4="TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_BUSY"
W=${WORKLOAD:-c3}
TO=${PASS_TIMEOUT:-60}
for K in ${KERNELS:-vcache_split}; do
i=0
for P in "$P0" "$P5" "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL $TO rocprofv3 --pmc $P -d gpurun_out/pmc_${W}_${K}_$i -o run --output-format csv -- python3 spmv-vector-cache_amd/tools/gpurun_pmc.py $K $W > gpurun_out/pmc_${W}_${K}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_${W}_${K}_$i.log; exit 1; }
  echo "pass $i ok"
done; done
echo done
