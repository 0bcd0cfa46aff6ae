cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/wgrad_group_probe.py > gpurun_out/r6c_probe.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/wgrad_group_probe.py layers=2 >> gpurun_out/r6c_probe.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/wgrad_group_probe.py layers=12 M=4096 D=768 >> gpurun_out/r6c_probe.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c_prof -o run --output-format csv -- python3 tools/wgrad_group_probe.py reps=5 > gpurun_out/r6c_prof.log 2>&1 || exit $?
bash tools/pmc_pass.sh r6c_pmc tools/wgrad_group_probe.py reps=5 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/r6c_pmc_p5 -o run -- python3 tools/wgrad_group_probe.py reps=5 > gpurun_out/r6c_pmc_p5.log 2>&1 || exit $?
echo done
