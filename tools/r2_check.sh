#!/bin/bash
# Round-2 GPU session: all -m gpu tests (one process per file), smoke(), the
# default bench line, rocprof kernel stats of a short bench, PMC passes of the
# roofline loop and of a short train step.  Every GPU step has its own time
# limit; the script stops at the first crash.  Usage: tools/r2_check.sh TAG [steps]
cd "$(dirname "$0")/.."
TAG=${1:-r2}; shift
STEPS=${@:-tests smoke bench prof pmc}
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in $STEPS; do
  case $s in
    tests) for f in tests/test_gpu_*.py; do
             b=$(basename $f .py)
             timeout -k 10 600 python -u -m pytest $f -q -m gpu -rf --timeout 300 --timeout-method thread \
               -p no:cacheprovider > gpurun_out/${TAG}_$b.log 2>&1
             rc=$?; tail -3 gpurun_out/${TAG}_$b.log
             if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $f exited $rc"; exit $rc; fi
           done ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $? ;;
    bench) timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $? ;;
    quick) timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_quick.log 2>&1 || exit $? ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
            python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || exit $? ;;
    roofprof) timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_roofprof -o run --output-format csv -- \
            python3 bench.py --roofline-only --roofline-op ${ROOFOP:-vit_linear_wgrad} > gpurun_out/${TAG}_roofprof.log 2>&1 || exit $? ;;
    pmc) bash tools/pmc_pass.sh ${TAG}_rpmc bench.py --roofline-only --roofline-op ${ROOFOP:-vit_linear_wgrad} || exit $? ;;
    large) timeout -k 10 300 python -u bench.py --variant large --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_large_bf16.log 2>&1 || exit $?
           timeout -k 10 300 python -u bench.py --variant large --attn fp8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_large_fp8.log 2>&1 || exit $?
           timeout -k 10 300 python -u bench.py --mode infer --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_infer.log 2>&1 || exit $? ;;
    pmcstep)bash tools/pmc_pass.sh ${TAG}_spmc bench.py --steps 2 --warmup 2 --no-cpu-baseline || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "step $s ok"
done
