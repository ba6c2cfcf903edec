cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for b in 16000000 32000000 16000000 32000000; do
  timeout -k 10 300 python bench.py --no-cpu --steps 6 --warmup 2 --batch $b > gpurun_out/batch_$b.json 2> gpurun_out/batch_$b.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/batch_$b.json'));r=d['roofline'];print('batch %s %.4e ph/s  step %.2f ms transport %.2f ms  fold %.2f ms launches %d' % ('$b', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['deposit_fold_ms_per_launch'], r['launches_timed']))"
done
