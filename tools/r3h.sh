cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3h_attn -o run --output-format csv -- python3 tools/attn_bench.py > gpurun_out/r3h_attn.log 2>&1 || exit 1
bash tools/pmc_attn2.sh r3hpmc
