#!/bin/bash
# rocprofv3 PMC passes (counters only: no trace domains) over the roofline
# kernel loop.  Usage: tools/pmc_pass.sh TAG
cd "$(dirname "$0")/.."
TAG=${1:-pmc}
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_p$i -o run -- \
    python3 bench.py --roofline-only > gpurun_out/${TAG}_p$i.log 2>&1 || exit $?
  echo "pass $i ok"
done
