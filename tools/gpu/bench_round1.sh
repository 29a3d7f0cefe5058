set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_fail; cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --cpu-seconds 5 > gpurun_out/bench_syn4.json 2> gpurun_out/bench_syn4.err || { echo bench_fail; tail gpurun_out/bench_syn4.err; exit 1; }
timeout -k 10 120 mpi_pastar_msa_amd/bin/msa_pastar tests/golden/PF08184.fasta > gpurun_out/cli_pf.txt 2>&1 || { echo cli_fail; cat gpurun_out/cli_pf.txt; exit 1; }
timeout -k 10 300 python bench.py --workload kinase --table-log2 26 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_kinase.json 2> gpurun_out/bench_kinase.err || { echo kin_fail; tail gpurun_out/bench_kinase.err; exit 1; }
timeout -k 10 400 python bench.py --workload syn8x400_s5 --table-log2 28 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_syn8.json 2> gpurun_out/bench_syn8.err || { echo syn8_fail; tail gpurun_out/bench_syn8.err; exit 1; }
cat gpurun_out/smoke.log gpurun_out/bench_syn4.json gpurun_out/cli_pf.txt gpurun_out/bench_kinase.json gpurun_out/bench_syn8.json
