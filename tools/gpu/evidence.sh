# Round evidence: GPU tests, smoke, bench lines of every workload (CPU legs
# for the three fast ones), then rocprofv3 traces and PMC passes per workload
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
rm -f gpurun_out/ev/partial_probe.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ev/tests.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/ev/tests.log; exit 1; }
tail -2 gpurun_out/ev/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev/smoke.log 2>&1 || { echo smoke_fail; exit 1; }
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/ev/bench_syn4x200_s1.json 2> gpurun_out/ev/b1.err || { echo bench_fail; tail gpurun_out/ev/b1.err; exit 1; }
timeout -k 10 300 python bench.py --workload PF08184 --steps 200 --warmup 20 > gpurun_out/ev/bench_PF08184.json 2> gpurun_out/ev/b2.err || { echo bench_fail; exit 1; }
timeout -k 10 300 python bench.py --workload kinase --steps 10 --warmup 2 --cpu-seconds 10 > gpurun_out/ev/bench_kinase.json 2> gpurun_out/ev/b3.err || { echo bench_fail; exit 1; }
timeout -k 10 300 python bench.py --workload syn8x400_s5 --steps 5 --warmup 1 --cpu-legs tN --cpu-seconds 30 > gpurun_out/ev/bench_syn8x400_s5.json 2> gpurun_out/ev/b4.err || { echo bench_fail; exit 1; }
timeout -k 10 200 python -u tools/gpu/probe_shards.py syn4x200_s1,kinase,syn8x400_s5 1,2,4,8 1 > gpurun_out/ev/sharded_one_gpu.txt 2>&1 || { echo shard_probe_fail; tail gpurun_out/ev/sharded_one_gpu.txt; exit 1; }
SHIFT=18 timeout -k 10 200 python -u tools/gpu/probe_shards.py syn4x200_s1,kinase 2,4,8 1 > gpurun_out/ev/sharded_one_gpu_shift18.txt 2>&1 || { echo shard_probe_fail; exit 1; }
timeout -k 10 200 python -u tools/gpu/many_probe.py > gpurun_out/ev/many_probe.txt 2>&1 || { echo many_probe_fail; exit 1; }
for k in -1 none; do if [ $k = none ]; then unset PASTAR_PARTIAL_K; else export PASTAR_PARTIAL_K=$k; fi; for w in syn8x400_s5 syn8x100_s3 syn8x400_s11; do timeout -k 10 100 python tools/gpu/partial_probe.py $w 4 >> gpurun_out/ev/partial_probe.txt 2>&1 || { echo partial_probe_fail; exit 1; }; done; done; unset PASTAR_PARTIAL_K
[ -f tools/gpu/libpastar_gpu_phases.so ] && { bash tools/gpu/phases.sh syn4x200_s1 3 > gpurun_out/ev/dive_phases.txt 2>&1 || { echo phases_fail; exit 1; }; }
bash tools/gpu/profile_all.sh syn4x200_s1 PF08184 kinase syn8x400_s5 > gpurun_out/ev/profile.log 2>&1 || { echo profile_fail; tail gpurun_out/ev/profile.log; exit 1; }
echo evidence_ok
