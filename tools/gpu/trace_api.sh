# HIP API + kernel trace of the syn8x400 bench (where does a step go?)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tr_${W:-syn8x400_s5}
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/tr_${W:-syn8x400_s5} -o run -- python3 bench.py --workload ${W:-syn8x400_s5} --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tr_${W:-syn8x400_s5}/bench.json 2> gpurun_out/tr_${W:-syn8x400_s5}/err.log || { echo fail; tail gpurun_out/tr_${W:-syn8x400_s5}/err.log; exit 1; }
head -12 gpurun_out/tr_${W:-syn8x400_s5}/run_hip_api_stats.csv
head -8 gpurun_out/tr_${W:-syn8x400_s5}/run_kernel_stats.csv
cat gpurun_out/tr_${W:-syn8x400_s5}/bench.json
