cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for f in 1.0 0.95 0.9 0.85 0.75; do
  SMCRT_GRID_FRAC=$f timeout -k 10 240 python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/frac_$f.json 2> gpurun_out/frac_$f.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/frac_$f.json'));r=d['roofline'];print('frac %s %.4e ph/s  step %.2f ms transport %.2f ms  fold %.2f ms' % ('$f', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['deposit_fold_ms_per_launch']))"
done
