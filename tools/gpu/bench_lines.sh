# the bench lines of every workload (after profiles/pmc_*.json are current)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/b_default.json 2> gpurun_out/b_default.err || { echo bench_fail; tail gpurun_out/b_default.err; exit 1; }
timeout -k 10 300 python bench.py --workload PF08184 --steps 20 --warmup 3 > gpurun_out/b_pf.json 2> gpurun_out/b_pf.err || { echo pf_fail; exit 1; }
timeout -k 10 300 python bench.py --workload kinase --steps 3 --warmup 1 > gpurun_out/b_kin.json 2> gpurun_out/b_kin.err || { echo kin_fail; exit 1; }
timeout -k 10 300 python bench.py --workload syn8x400_s5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_syn8.json 2> gpurun_out/b_syn8.err || { echo syn8_fail; exit 1; }
cat gpurun_out/b_default.json
