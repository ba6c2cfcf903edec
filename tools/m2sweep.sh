cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
for b in 6400000 25600000 51200000; do
  WL=m2 BATCH=$b STEPS=4 bash tools/exp_env.sh || exit 1
done
WL=m5 STEPS=8 bash tools/exp_env.sh && WL=m4 STEPS=4 bash tools/exp_env.sh
