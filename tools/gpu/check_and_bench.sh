# parity tests (search subset) + bench lines on the main workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q --timeout=300 -k "search or random" > gpurun_out/t_search.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/t_search.log; exit 1; }
tail -3 gpurun_out/t_search.log
timeout -k 10 300 python bench.py --cpu-seconds 5 > gpurun_out/b_syn4.json 2> gpurun_out/b_syn4.err || { echo b1_fail; tail gpurun_out/b_syn4.err; exit 1; }
timeout -k 10 300 python bench.py --workload kinase --table-log2 26 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_kin.json 2> gpurun_out/b_kin.err || { echo b2_fail; tail gpurun_out/b_kin.err; exit 1; }
timeout -k 10 400 python bench.py --workload syn8x400_s5 --table-log2 28 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_syn8.json 2> gpurun_out/b_syn8.err || { echo b3_fail; tail gpurun_out/b_syn8.err; exit 1; }
for f in b_syn4 b_kin b_syn8; do python -c "
import json;d=json.load(open('gpurun_out/$f.json'));r=d['roofline']
print('$f', 'value %.3g'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'wall %.4f'%d['wall_to_optimal_s'], 'exp %d'%d['expansions_per_search'], 'ok',d['score_ok'], 'frac %.4f'%r['frac'], 'avg_us %.1f'%r['avg_launch_us'], 'launches', r['launches'], 'cpu', d.get('cpu_baseline',{}).get('value'))"; done
