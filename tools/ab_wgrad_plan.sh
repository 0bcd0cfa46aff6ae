set -o pipefail
for i in 1 2; do
  for p in 0 1; do
    timeout -k 10 300 python -u tools/bench_tune.py 6=$p -- --no-cpu-baseline > gpurun_out/r6e_plan${p}_$i.log 2>&1 || exit $?
    python -c "import json,sys;l=[x for x in open('gpurun_out/r6e_plan${p}_$i.log') if x.startswith('{')][-1];d=json.loads(l);t=d['op_table'];print('plan $p run $i', d['ms_per_step'], 'wgrad', t['vit_linear_wgrad']['ms_per_step'], 'dgrad', t['vit_linear_dgrad']['ms_per_step'])"
  done
done
