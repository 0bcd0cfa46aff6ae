#!/bin/bash
# End-of-round GPU evidence in one call: every -m gpu test file, smoke(), the
# default bench line (with the CPU baseline), rocprof kernel statistics of a
# short bench and of the roofline loop, and the PMC passes of the roofline
# kernel.  Each GPU step has its own time limit; the script stops at the first
# failure.  Usage: tools/final_check.sh TAG
cd "$(dirname "$0")/.."
TAG=${1:-final}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_train_step.py \
  tests/test_gpu_enhancer.py > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
grep -q "failed" gpurun_out/test_gpu_*.log && { echo "test failures"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_roofprof -o run --output-format csv -- \
  python3 bench.py --roofline-only > gpurun_out/${TAG}_roofprof.log 2>&1 || exit $?
bash tools/pmc_pass.sh ${TAG}_pmc || exit $?
echo "final check ok"
