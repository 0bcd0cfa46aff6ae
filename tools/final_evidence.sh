#!/bin/bash
# Final evidence of a round: the whole -m gpu suite in one process (as the
# driver runs it), the default bench line (graph mode, CPU baseline), the
# config-2 / config-5 lines, rocprofv3 kernel stats of a short bench, and the
# ViT forward / data-gradient classes re-run in isolation under rocprofv3
# (--kernel-trace --stats) with their FETCH_SIZE / WRITE_SIZE PMC passes
# (tools/roofline_pmc.py turns those into profiles/roofline_pmc.json).
# Usage: tools/final_evidence.sh TAG
cd "$(dirname "$0")/.."
TAG=${1:-r6f}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: GPU tests exited $rc"; exit $rc; fi
bash tools/gpu_session.sh $TAG bench infer large largefp8 prof roof:vit_linear_fwd roof:vit_linear_dgrad || exit $?
