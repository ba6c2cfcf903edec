set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh
rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload m5 --batch 16000000 --steps 2 --warmup 1 --no-cpu > gpurun_out/m5_16M.json 2> gpurun_out/m5_16M.err
echo "m5 rc=$?"; cat gpurun_out/m5_16M.json
