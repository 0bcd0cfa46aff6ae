#!/bin/bash
# Counter passes over tools/attn_bench.py (attention fwd / bwd at the B=32 shape):
# instruction mix (VALU / MFMA / LDS / SALU / VMEM), active and wait cycles.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-attn}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_p$i -o run -- \
    python3 tools/attn_bench.py > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
