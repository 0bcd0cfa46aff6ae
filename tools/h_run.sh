#!/bin/bash
# Iteration run: GPU tests of the given files (default kernels+model+train step),
# the conv/attention probes and a quick bench.  Usage: tools/h_run.sh TAG [test files]
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-h}; shift
FILES=${@:-tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_train_step.py}
timeout -k 10 400 python -u -m pytest $FILES -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG}_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 100 python -u tools/conv_probe.py > gpurun_out/${TAG}_conv.log 2>&1 && cat gpurun_out/${TAG}_conv.log &&
timeout -k 10 100 python -u tools/attn_sweep.py > gpurun_out/${TAG}_attn.log 2>&1 && cat gpurun_out/${TAG}_attn.log &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_quick.log 2>&1 &&
python tools/opt.py gpurun_out/${TAG}_quick.log
