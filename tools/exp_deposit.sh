cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in default NO_ATOMIC; do
  if [ $v = default ]; then export SMCRT_LIB=""; else export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_$v.so; fi
  timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/exp.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/exp.json'));print('$v', '%.3e'%d['value'], d['roofline']['avg_launch_ms'])"
done
