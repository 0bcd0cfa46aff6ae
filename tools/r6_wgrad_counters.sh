#!/bin/bash
# Verdict r5 item 1's counter pass, before / after: the ViT weight-gradient class
# of one B=32 step re-run in isolation (bench.py --roofline-only) as the per-Linear
# split-K launches (HF.WGRAD_GROUP=0, the round-5 path) and as the grouped launch,
# each under two rocprofv3 --pmc passes (SQ, then TCC; no tracing in the same run).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r6cnt}
for g in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY \
    --output-format csv -d gpurun_out/${TAG}_g${g}_sq -o run -- \
    python3 tools/bench_tune.py HF.WGRAD_GROUP=$g -- --roofline-only --roofline-op vit_linear_wgrad \
    > gpurun_out/${TAG}_g${g}_sq.log 2>&1 || exit $?
  echo "step g$g sq ok"
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
    --output-format csv -d gpurun_out/${TAG}_g${g}_tcc -o run -- \
    python3 tools/bench_tune.py HF.WGRAD_GROUP=$g -- --roofline-only --roofline-op vit_linear_wgrad \
    > gpurun_out/${TAG}_g${g}_tcc.log 2>&1 || exit $?
  echo "step g$g tcc ok"
done
