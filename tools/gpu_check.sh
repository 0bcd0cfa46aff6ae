#!/bin/bash
# One GPU-box session: parity tests, GEMM micro-bench, short bench, rocprof
# kernel statistics.  Every GPU step has its own time limit and the script
# stops at the first failure.  Usage: tools/gpu_check.sh TAG [steps...]
# steps: tests gemm bench prof (default: all)
cd "$(dirname "$0")/.."
TAG=${1:-run}; shift
STEPS=${@:-tests gemm bench prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests) bash tools/gpu_tests.sh tests/test_gpu_kernels.py tests/test_gpu_model.py > gpurun_out/${TAG}_tests.log 2>&1 || exit $? ;;
    gemm) timeout -k 10 240 python tools/gemm_bench.py > gpurun_out/${TAG}_gemm.log 2>&1 || exit $? ;;
    stamps) HVIT_LIB=libhvit_stamps.so timeout -k 10 120 python tools/gemm_stamps.py > gpurun_out/${TAG}_stamps.log 2>&1 || exit $? ;;
    attn) timeout -k 10 120 python tools/attn_bench.py > gpurun_out/${TAG}_attn.log 2>&1 || exit $? ;;
    probe) timeout -k 10 240 python tools/gemm_probe.py > gpurun_out/${TAG}_probe.log 2>&1 || exit $? ;;
    bench) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || exit $? ;;
    fullbench) timeout -k 10 400 python bench.py > gpurun_out/${TAG}_fullbench.log 2>&1 || exit $? ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "step $s ok"
done
