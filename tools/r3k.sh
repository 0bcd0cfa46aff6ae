cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "mhsa" --timeout 120 > gpurun_out/r3k_attn_test.log 2>&1; tail -2 gpurun_out/r3k_attn_test.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3k_attn -o run --output-format csv -- python3 tools/attn_bench.py > gpurun_out/r3k_attn.log 2>&1 || exit 1
bash tools/r3_check.sh r3k tests:tests/test_gpu_dp.py bench prof
