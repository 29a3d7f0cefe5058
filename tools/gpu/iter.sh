# iteration loop on the GPU box: GPU tests, then the three bench workloads,
# then a kernel-trace of the default bench (summary under gpurun_out/iter_prof)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q --timeout=300 > gpurun_out/t_all.log 2>&1 || { echo tests_fail; tail -40 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --cpu-seconds 3 > gpurun_out/b_default.json 2> gpurun_out/b_default.err || { echo bench_fail; tail gpurun_out/b_default.err; exit 1; }
timeout -k 10 300 python bench.py --workload kinase --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_kin.json 2> gpurun_out/b_kin.err || { echo kin_fail; tail gpurun_out/b_kin.err; exit 1; }
timeout -k 10 300 python bench.py --workload syn8x400_s5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_syn8.json 2> gpurun_out/b_syn8.err || { echo syn8_fail; tail gpurun_out/b_syn8.err; exit 1; }
timeout -k 10 300 python bench.py --workload PF08184 --steps 20 --warmup 3 --cpu-seconds 3 > gpurun_out/b_pf.json 2> gpurun_out/b_pf.err || { echo pf_fail; tail gpurun_out/b_pf.err; exit 1; }
for f in b_default b_kin b_syn8 b_pf; do
python -c "
import json,sys;d=json.load(open('gpurun_out/$f.json'));r=d['roofline']
print('$f', d['config']['workload'], 'value %.3g ms/step %.2f wall %.4f exp %d steps %.0f graph %s avg_us %.1f (sel %.1f gap %.1f) frac %.4f score_ok %s'%(d['value'],d['ms_per_step'],d['wall_to_optimal_s'],d['expansions_per_search'],d['steps_per_search'],d['graph_replay'],r['avg_launch_us'],r['avg_select_tail_us'],r['avg_gap_us'],r['frac'],d['score_ok']), 'cpu %.3g'%d['cpu_baseline']['value'] if 'cpu_baseline' in d else '')"
done
mkdir -p gpurun_out/iter_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/iter_prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/iter_prof/bench.json 2> gpurun_out/iter_prof/err.log || { echo prof_fail; tail gpurun_out/iter_prof/err.log; exit 1; }
head -6 gpurun_out/iter_prof/run_kernel_stats.csv
