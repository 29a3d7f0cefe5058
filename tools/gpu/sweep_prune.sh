# bench.py lines of a workload with the children pruned at a given upper
# bound of the optimum (PASTAR_PRUNE_F = optimum + delta): what a bound of
# that quality is worth.  usage: bash tools/gpu/sweep_prune.sh workload optimum "deltas..." [steps]
set -o pipefail
cd $GRAFT_REPO_ROOT
W=$1; C=$2; DS=$3; S=${4:-3}
for d in $DS; do
  if [ $d = none ]; then unset PASTAR_PRUNE_F; else export PASTAR_PRUNE_F=$((C + d)); fi
  timeout -k 10 120 python bench.py --workload $W --steps $S --warmup 2 --no-cpu-baseline --no-north-star --no-sub-records > gpurun_out/sw.json 2>gpurun_out/sw.err || { echo sweep_fail $d; tail gpurun_out/sw.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('delta=$d $W ms/step %.3f loop %.3f exp %d steps %.1f launch %.1f us children %.0f ok %s' % (d['ms_per_step'], d['search_loop_s']*1e3, d['expansions_per_search'], d['steps_per_search'], d['roofline']['avg_launch_us'], d['roofline']['probes']['children_per_search'], d['score_ok']))"
done
