#!/bin/bash
# PMC passes (one small counter group per rocprofv3 run, kernel-trace only --
# never combined with sys/runtime traces) over the product kernel in bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/pmc; mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--kernel vcache_split --mode fast --steps 10 --warmup 3 --no-cpu-baseline --no-rocprof"}
GROUPS_DEFAULT="FETCH_SIZE WRITE_SIZE TCC_HIT_sum,TCC_MISS_sum SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY"
read -r -a GROUPS_ARR <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
i=0
for grp in "${GROUPS_ARR[@]}"; do
  i=$((i+1))
  ctrs=${grp//,/ }
  echo "== pass $i: $ctrs"
  timeout -k 10 120 rocprofv3 --pmc $ctrs -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
find $OUT -name "*counter_collection.csv" | sort
