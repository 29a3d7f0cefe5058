# expand grid cap sweep (PASTAR_EXPAND_BLOCKS) on the throughput workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests -m gpu -x -q --timeout=200 > gpurun_out/t_all.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
for B in ${BLOCKS:-0}; do
  echo "== blocks $B"
  if [ $B = 0 ]; then unset PASTAR_EXPAND_BLOCKS; else export PASTAR_EXPAND_BLOCKS=$B; fi
  timeout -k 10 120 python tools/gpu/probe.py ${WL:-kinase,syn8x400_s5,syn4x200_s1} 3 || exit 1
done
