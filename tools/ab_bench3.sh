#!/bin/bash
# In-step A/B on one box: old library, ring off, ring auto (bench.py --no-cpu-baseline), alternating.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-ab}
for r in 1 2; do
  HVIT_LIB=libhvit_old.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/${TAG}_old_$r.log 2>&1 || exit $?
  HVIT_RING=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/${TAG}_r0_$r.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/${TAG}_auto_$r.log 2>&1 || exit $?
done
python3 - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{tag}_*.log")):
    l = [x for x in open(f) if x.startswith("{")][-1]
    d = json.loads(l)
    ops = {k: v["ms_per_step"] for k, v in d["op_table"].items()}
    print(f.split("/")[-1], d["ms_per_step"], d["ms_per_step_median"], {k: ops[k] for k in list(ops)[:7]})
PY
