#!/bin/bash
# PMC passes over the attention micro-benchmark (counters only, no traces)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || exit $?
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU" ; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $set --output-format csv -d gpurun_out/attnpmc_p$i -o run -- \
    python3 tools/attn_bench.py > gpurun_out/attnpmc_p$i.log 2>&1 || exit $?
  echo "pass $i ok"
done
