#!/bin/bash
# GPU-box session: steps run in order, each under its own time limit; the
# script stops at the first crash / timeout.  Usage: tools/gpu_session.sh TAG step...
#   tests[:file,...]  GPU test files (default: all tests/test_gpu_*.py)
#   bench             default bench.py line (graph mode, CPU baseline)
#   benchq            bench.py without the CPU baseline
#   eager             bench.py --graph 0 --no-cpu-baseline
#   dp1               bench.py's DP branch (RCCL, GradAllReducer, captured step) at world 1 under torchrun
#   roof:OP           op class OP re-run in isolation: rocprofv3 kernel stats and FETCH/WRITE_SIZE passes
#   infer             bench.py --mode infer (BASELINE config 2)
#   large / largefp8  bench.py --variant large [--attn fp8] (BASELINE config 5)
#   prof              rocprofv3 kernel stats of a short bench
#   gemm              tools/gemm_bench.py
#   env:VAR=VAL,...   benchq under extra environment variables (A/B knobs)
#   py:SCRIPT[:ARGS]  python SCRIPT ARGS (a probe under tools/; ARGS space-separated by '+')
cd "$(dirname "$0")/.."
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in "$@"; do
  case $s in
    tests*)
      files=${s#tests}; files=${files#:}
      if [ -z "$files" ]; then files=$(ls tests/test_gpu_*.py); else files=$(echo $files | tr ',' ' '); fi
      for f in $files; do
        timeout -k 10 900 python -u -m pytest "$f" -q -m gpu -rf --maxfail=40 -p no:cacheprovider \
          --timeout 300 --timeout-method thread > "gpurun_out/${TAG}_$(basename $f .py).log" 2>&1
        rc=$?
        tail -5 "gpurun_out/${TAG}_$(basename $f .py).log"
        if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $f exited $rc"; exit $rc; fi
      done ;;
    bench) timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $? ;;
    benchq) timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_benchq.log 2>&1 || exit $? ;;
    infer) timeout -k 10 400 python -u bench.py --mode infer --no-cpu-baseline > gpurun_out/${TAG}_infer.log 2>&1 || exit $? ;;
    large) timeout -k 10 400 python -u bench.py --variant large --no-cpu-baseline > gpurun_out/${TAG}_large.log 2>&1 || exit $? ;;
    largefp8) timeout -k 10 400 python -u bench.py --variant large --attn fp8 --no-cpu-baseline > gpurun_out/${TAG}_largefp8.log 2>&1 || exit $? ;;
    eager) timeout -k 10 400 python -u bench.py --graph 0 --no-cpu-baseline > gpurun_out/${TAG}_eager.log 2>&1 || exit $? ;;
    dp1) HVIT_FORCE_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
           --master-addr 127.0.0.1 --master-port 29531 bench.py --no-cpu-baseline > gpurun_out/${TAG}_dp1.log 2>&1 || exit $? ;;
    roof:*)  # roof:OP -- the op class re-run in isolation: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes
      op=${s#roof:}
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_roofprof_$op -o run --output-format csv -- \
        python3 bench.py --roofline-only --roofline-op $op > gpurun_out/${TAG}_roofprof_$op.log 2>&1 || exit $?
      for set in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_rpmc_${op}_$set -o run -- \
          python3 bench.py --roofline-only --roofline-op $op > gpurun_out/${TAG}_rpmc_${op}_$set.log 2>&1 || exit $?
      done ;;
    prof) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || exit $? ;;
    env:*)  # env:VAR=VAL[,VAR=VAL]: bench.py --no-cpu-baseline under those variables
      kv=${s#env:}; tagv=$(echo "$kv" | tr ',=' '__')
      env $(echo "$kv" | tr ',' ' ') timeout -k 10 400 python -u bench.py --no-cpu-baseline \
        > gpurun_out/${TAG}_env_${tagv}.log 2>&1 || exit $? ;;
    py:*)
      spec=${s#py:}; script=${spec%%:*}; args=""; [ "$spec" != "$script" ] && args=$(echo "${spec#*:}" | tr '+' ' ')
      timeout -k 10 300 python -u $script $args > gpurun_out/${TAG}_$(basename $script .py).log 2>&1 || exit $? ;;
    gemm) timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/${TAG}_gemm.log 2>&1 || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "step $s ok"
done
