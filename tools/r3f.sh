cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_exact.py -q -k "small" --timeout 120 > gpurun_out/r3f_ws_test.log 2>&1; tail -2 gpurun_out/r3f_ws_test.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3f_ws -o run --output-format csv -- python3 tools/wgrad_small.py > gpurun_out/r3f_ws.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3f_probe -o run --output-format csv -- python3 tools/c1_probe.py reps=5 > gpurun_out/r3f_probe.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py -q -s --timeout 600 -k "batch32_train or eval_forward or batch32_eval" > gpurun_out/r3f_model.log 2>&1; tail -2 gpurun_out/r3f_model.log
timeout -k 10 300 python bench.py --mode infer --no-cpu-baseline > gpurun_out/r3f_infer1.log 2>&1 || exit 1
HVIT_EVALFOLD=0 timeout -k 10 300 python bench.py --mode infer --no-cpu-baseline > gpurun_out/r3f_infer0.log 2>&1 || exit 1
bash tools/r3_check.sh r3f prof
