#!/bin/bash
# Final evidence of a round: every GPU test file, the default bench line (graph
# mode, CPU baseline), the config-2 / config-5 lines, rocprofv3 kernel stats of a
# short bench, the dominant op class re-run in isolation under rocprofv3
# (--kernel-trace --stats) and its FETCH_SIZE / WRITE_SIZE PMC passes.
# Usage: tools/final_evidence.sh TAG [OP]
cd "$(dirname "$0")/.."
TAG=${1:-r3f}; OP=${2:-vit_linear_dgrad}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_session.sh $TAG tests bench infer large largefp8 prof || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_roofprof -o run --output-format csv -- \
  python3 bench.py --roofline-only --roofline-op $OP > gpurun_out/${TAG}_roofprof.log 2>&1 || exit $?
echo "step roofprof ok"
for set in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_rpmc_$set -o run -- \
    python3 bench.py --roofline-only --roofline-op $OP > gpurun_out/${TAG}_rpmc_$set.log 2>&1 || exit $?
  echo "step pmc $set ok"
done
