set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q --timeout=300 > gpurun_out/t_all.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 200 python tools/tune.py syn4x200_s1 --mult 0.25,0.5,1 --batch 32768 > gpurun_out/tune_syn4.txt 2>&1; echo rc=$?
timeout -k 10 300 python tools/tune.py kinase --mult 0.25,0.5 --batch 32768 --reps 1 > gpurun_out/tune_kin.txt 2>&1; echo rc=$?
timeout -k 10 300 python tools/tune.py syn8x400_s5 --mult 0.25 --batch 32768 --reps 1 --table-log2 28 > gpurun_out/tune_syn8.txt 2>&1; echo rc=$?
timeout -k 10 300 python bench.py --cpu-seconds 3 > gpurun_out/b_default.json 2> gpurun_out/b_default.err || { echo bench_fail; tail gpurun_out/b_default.err; exit 1; }
cat gpurun_out/tune_syn4.txt gpurun_out/tune_kin.txt gpurun_out/tune_syn8.txt
python -c "
import json;d=json.load(open('gpurun_out/b_default.json'));r=d['roofline']
print('BENCH value %.3g ms/step %.2f wall %.4f exp %d steps %.0f graph %s avg_us %.1f launches %d cpu %.3g'%(d['value'],d['ms_per_step'],d['wall_to_optimal_s'],d['expansions_per_search'],d['steps_per_search'],d['graph_replay'],r['avg_launch_us'],r['launches'],d['cpu_baseline']['value']))"
