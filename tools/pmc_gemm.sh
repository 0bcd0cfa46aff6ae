#!/bin/bash
# PMC passes over the GEMM micro-benchmark (counters only, no traces)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES" ; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d gpurun_out/gemmpmc_p$i -o run -- \
    python3 tools/gemm_bench.py > gpurun_out/gemmpmc_p$i.log 2>&1 || exit $?
  echo "pass $i ok"
done
