#!/bin/bash
# rocprofv3 PMC passes (counters only: no trace domains), one run per counter
# set, over a command (default: the dominant op's loop, bench.py --roofline-only).
# Usage: tools/pmc_pass.sh TAG [python3 args...]
cd "$(dirname "$0")/.."
TAG=${1:-pmc}; shift
ARGS=${@:-bench.py --roofline-only}
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_p$i -o run -- \
    python3 $ARGS > gpurun_out/${TAG}_p$i.log 2>&1 || exit $?
  echo "pass $i ok"
done
