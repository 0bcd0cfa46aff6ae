# A/B of the Cout = 1 forward forms (HVIT_O1F_FORM 1: chunk lanes + shuffles, 2: thread per pixel)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "1 128" "2 128" "2 256"; do
  set -- $cfg
  HVIT_O1F_FORM=$1 HVIT_O1F_PIX=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/o1ab2_$1_$2 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/o1ab2_$1_$2.log 2>&1 || exit $?
done
