cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_c1block.py -q -x --timeout 120 > gpurun_out/c1e_test.log 2>&1; tail -2 gpurun_out/c1e_test.log
timeout -k 10 120 python tools/wgrad_small.py > gpurun_out/ws_default.log 2>&1 || exit 1
HVIT_NO_RS=1 timeout -k 10 120 python tools/wgrad_small.py > gpurun_out/ws_nors.log 2>&1 || exit 1
timeout -k 10 200 python tools/c1_probe.py mfma=1 > gpurun_out/c1p_1.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py -q -s --timeout 400 > gpurun_out/sg_test.log 2>&1; tail -2 gpurun_out/sg_test.log
bash tools/r3_check.sh sg env:HVIT_SKIPGRAD=0 env:HVIT_SKIPGRAD=1 || exit 1
timeout -k 10 300 python bench.py --mode infer --no-cpu-baseline > gpurun_out/sg_infer1.log 2>&1 || exit 1
HVIT_EVALFOLD=0 timeout -k 10 300 python bench.py --mode infer --no-cpu-baseline > gpurun_out/sg_infer0.log 2>&1
