# rocprofv3 kernel stats of the syn4x200 bench under the two-step and the
# one-step backtrace walk (PASTAR_WALK1); prints the walk kernels' rows
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 0 1; do
  PASTAR_WALK1=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/walk_$v -o p --output-format csv -- python3 bench.py --workload ${1:-syn4x200_s1} --steps 20 --warmup 5 --no-cpu-baseline --no-north-star > gpurun_out/walk_$v.log 2>&1 || { echo prof_fail; tail gpurun_out/walk_$v.log; exit 1; }
  echo "PASTAR_WALK1=$v"; grep -h "walk\|tail_pack\|census\|copyBuffer\|search_init" gpurun_out/walk_$v/p_kernel_stats.csv | cut -c1-200
done
