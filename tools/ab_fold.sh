cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_ab.log; [ $rc -ne 0 ] && exit $rc
for mode in sync async sync async; do
  extra=""; [ $mode = sync ] && extra="--sync-fold"
  timeout -k 10 240 python bench.py --no-cpu --steps 10 --warmup 2 $extra > gpurun_out/ab_$mode.json 2> gpurun_out/ab_$mode.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$mode.json'));r=d['roofline'];print('%-6s %.4e ph/s  step %.2f ms transport %.2f ms  fold %.2f ms' % ('$mode', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['deposit_fold_ms_per_launch']))"
done
