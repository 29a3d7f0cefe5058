# like sweep_env.sh, with --no-sub-records and the child (probe) count; usage:
# bash tools/gpu/sweep_env2.sh VAR "v1 v2 ..." [workload] [steps]   (value "none": variable unset)
set -o pipefail
cd $GRAFT_REPO_ROOT
VAR=$1; VALS=$2; W=${3:-syn8x400_s5}; S=${4:-3}
for v in $VALS; do
  if [ $v = none ]; then unset $VAR; else export $VAR=$v; fi
  timeout -k 10 300 python bench.py --workload $W --steps $S --warmup 2 --no-cpu-baseline --no-north-star --no-sub-records > gpurun_out/sw.json 2>gpurun_out/sw.err || { echo sweep_fail $v; tail gpurun_out/sw.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('$VAR=$v $W ms/step %.3f loop %.3f exp %d steps %.1f launch %.1f us children %.0f ok %s' % (d['ms_per_step'], d['search_loop_s']*1e3, d['expansions_per_search'], d['steps_per_search'], d['roofline']['avg_launch_us'], d['roofline']['probes']['children_per_search'], d['score_ok']))"
done
