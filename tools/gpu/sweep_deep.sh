# bench.py lines of a workload over PASTAR_DEEP_ROUNDS x --depth (block-local
# continuation on thin batches); usage: bash tools/gpu/sweep_deep.sh [workload] "rounds..." "depths..." [steps]
set -o pipefail
cd $GRAFT_REPO_ROOT
W=${1:-syn8x400_s5}; RS=${2:-"1 4"}; DS=${3:-"4 8 16"}; S=${4:-3}
for r in $RS; do for d in $DS; do
  PASTAR_DEEP_ROUNDS=$r timeout -k 10 120 python bench.py --workload $W --steps $S --warmup 2 --depth $d --no-cpu-baseline --no-north-star --no-sub-records > gpurun_out/sw.json 2>gpurun_out/sw.err || { echo sweep_fail $r $d; tail gpurun_out/sw.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('rounds=$r depth=$d $W ms/step %.3f loop %.3f exp %d steps %.1f launch %.1f us ok %s' % (d['ms_per_step'], d['search_loop_s']*1e3, d['expansions_per_search'], d['steps_per_search'], d['roofline']['avg_launch_us'], d['score_ok']))"
done; done
