#!/bin/bash
# PMC passes over tools/ring_bench.py for one GEMM case and config:
#   tools/pmc_ring.sh TAG "only=<case substring>" cfgs=<c>
cd "$(dirname "$0")/.."
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for set in "TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
           "FETCH_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_p$i -o run -- \
    python3 tools/ring_bench.py check=0 rounds=1 "$@" > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
