# End-of-iteration evidence: GPU tests, smoke, the bench lines of every
# workload, then rocprofv3 kernel-trace + FETCH_SIZE / WRITE_SIZE passes
# (tools/gpu/profile_all.sh); summarised on the CPU side by tools/pmc_summary.py
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_fail; tail gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/b_default.json 2> gpurun_out/b_default.err || { echo bench_fail; tail gpurun_out/b_default.err; exit 1; }
timeout -k 10 300 python bench.py --workload PF08184 --steps 20 --warmup 3 > gpurun_out/b_pf.json 2> gpurun_out/b_pf.err || { echo pf_fail; exit 1; }
timeout -k 10 300 python bench.py --workload kinase --steps 3 --warmup 1 > gpurun_out/b_kin.json 2> gpurun_out/b_kin.err || { echo kin_fail; exit 1; }
timeout -k 10 300 python bench.py --workload syn8x400_s5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_syn8.json 2> gpurun_out/b_syn8.err || { echo syn8_fail; exit 1; }
cat gpurun_out/b_default.json
bash tools/gpu/profile_all.sh syn4x200_s1 PF08184 kinase syn8x400_s5
