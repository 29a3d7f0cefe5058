# bench.py lines of a workload under each value of one bench.py option;
# usage: bash tools/gpu/sweep_arg.sh --option "v1 v2 ..." [workload] [steps]
set -o pipefail
cd $GRAFT_REPO_ROOT
OPT=$1; VALS=$2; W=${3:-syn4x200_s1}; S=${4:-30}
for v in $VALS; do
  timeout -k 10 300 python bench.py --workload $W --steps $S --warmup 3 $OPT $v --no-cpu-baseline --no-north-star --no-sub-records > gpurun_out/sw.json 2>gpurun_out/sw.err || { echo sweep_fail $v; tail gpurun_out/sw.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('$OPT $v $W ms/step %.3f loop %.3f exp %d steps %.1f launch %.1f us ok %s' % (d['ms_per_step'], d['search_loop_s']*1e3, d['expansions_per_search'], d['steps_per_search'], d['roofline']['avg_launch_us'], d['score_ok']))"
done
