# bench.py lines of a workload under each --batch (parents per step)
set -o pipefail
cd $GRAFT_REPO_ROOT
VALS=$1; W=${2:-kinase}; S=${3:-6}
for v in $VALS; do
  timeout -k 10 300 python bench.py --workload $W --steps $S --warmup 2 --batch $v --no-cpu-baseline --no-north-star > gpurun_out/sw.json 2>gpurun_out/sw.err || { echo sweep_fail $v; tail gpurun_out/sw.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('batch=$v $W ms/step %.3f loop %.3f exp %d steps %.1f launch %.1f us' % (d['ms_per_step'], d['search_loop_s']*1e3, d['expansions_per_search'], d['steps_per_search'], d['roofline']['avg_launch_us']))"
done
