export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_train_step.py -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/h1_tests.log 2>&1; rc=$?; tail -5 gpurun_out/h1_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 100 python -u tools/attn_sweep.py > gpurun_out/h1_attn.log 2>&1 && cat gpurun_out/h1_attn.log &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/h1_quick.log 2>&1 && tail -c 600 gpurun_out/h1_quick.log
