#!/bin/bash
# PMC passes over tools/c1_probe.py: tools/pmc_c1.sh TAG [probe args]
cd "$(dirname "$0")/.."
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_p$i -o run -- \
    python3 tools/c1_probe.py reps=3 "$@" > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
