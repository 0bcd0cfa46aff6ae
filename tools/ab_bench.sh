#!/bin/bash
# A/B of env-selected variants on the quick bench, interleaved in one session.
# Usage: tools/ab_bench.sh TAG "ENV_A" "ENV_B" [...]   (each arg: space-separated VAR=VAL, or "-")
cd "$(dirname "$0")/.."
TAG=$1; shift
mkdir -p gpurun_out
i=0
for round in 1 2; do
  for v in "$@"; do
    i=$((i+1))
    envs=""; [ "$v" != "-" ] && envs="$v"
    env $envs timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_$i.log 2>&1 || exit $?
    python - "$v" gpurun_out/${TAG}_$i.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ops = " ".join(f"{k}={v['ms_per_step']:.3f}" for k, v in d["op_table"].items())
print(f"[{sys.argv[1]}] {d['ms_per_step']:.3f} ms/step | {ops}")
PY
  done
done
