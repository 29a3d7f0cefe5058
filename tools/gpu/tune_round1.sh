set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q --timeout=300 -k "search or random or autogrow" > gpurun_out/t_search.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/t_search.log; exit 1; }
tail -2 gpurun_out/t_search.log
timeout -k 10 200 python tools/tune.py syn4x200_s1 --mult 0.125,0.25,0.5,1 --batch 1024,8192 > gpurun_out/tune_syn4.txt 2>&1; echo rc=$?
timeout -k 10 300 python tools/tune.py kinase --mult 0.125,0.25,0.5 --batch 8192,32768 --reps 1 > gpurun_out/tune_kin.txt 2>&1; echo rc=$?
timeout -k 10 500 python tools/tune.py syn8x400_s5 --mult 0.125,0.25,0.5 --batch 8192,32768 --reps 1 --table-log2 28 > gpurun_out/tune_syn8.txt 2>&1; echo rc=$?
cat gpurun_out/tune_syn4.txt gpurun_out/tune_kin.txt gpurun_out/tune_syn8.txt
