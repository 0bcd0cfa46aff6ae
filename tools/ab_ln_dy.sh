#!/bin/bash
# A/B of functional.LN_DY_LOW (bf16 vs f32 gradient at the LayerNorm outputs), alternating, same box
set -o pipefail
cd "$(dirname "$0")/.."
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python -u tools/bench_tune.py HF.LN_DY_LOW=$v -- --no-cpu-baseline > gpurun_out/r6f_lndy${v}_$i.log 2>&1 || exit $?
    python -c "import json;l=[x for x in open('gpurun_out/r6f_lndy${v}_$i.log') if x.startswith('{')][-1];d=json.loads(l);t=d['op_table'];print('LN_DY_LOW=$v run $i', d['ms_per_step'], 'ln_bwd', t['layernorm_bwd']['ms_per_step'], 'dgrad', t['vit_linear_dgrad']['ms_per_step'])"
  done
done
