cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_exact.py -q -k "small" --timeout 120 > gpurun_out/r3g_ws_test.log 2>&1; tail -2 gpurun_out/r3g_ws_test.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g_ws -o run --output-format csv -- python3 tools/wgrad_small.py > gpurun_out/r3g_ws.log 2>&1 || exit 1
bash tools/pmc_c1.sh r3gc1
