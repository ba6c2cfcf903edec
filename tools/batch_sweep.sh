#!/bin/bash
# On the GPU box: bench the default library at several per-step batch sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for b in ${BATCHES:-4000000 8000000 16000000}; do
  timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS:-5} --warmup 2 --batch $b > gpurun_out/batch_$b.json 2> gpurun_out/batch_$b.err
  rc=$?; if [ $rc -ne 0 ]; then echo "batch $b rc=$rc"; tail -5 gpurun_out/batch_$b.err; exit $rc; fi
  python3 -c "import json;d=json.load(open('gpurun_out/batch_$b.json'));r=d['roofline'];print('batch %-10s %.4e ph/s  step %.1f ms  transport %.2f ms x%d  fold %.2f ms (chip)  iters %.3g' % ('$b', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['launches_timed'], r['fold_cu_ms_per_launch'], r['wave_iterations_per_launch']))"
done
