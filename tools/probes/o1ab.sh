# Pixels per workgroup of the Cout = 1 strip forward (HVIT_O1F_PIX), kernel stats per setting
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for px in 128 256; do
  HVIT_O1F_PIX=$px timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/o1ab3_$px -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/o1ab3_$px.log 2>&1 || exit $?
done
