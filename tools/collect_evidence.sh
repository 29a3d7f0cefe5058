# After `gpurun -- 'bash tools/gpu/evidence.sh'`: summarise what came back
# under gpurun_out/ into profiles/ (run on the CPU side, from the repo root).
# usage: bash tools/collect_evidence.sh [round tag, default r3]
set -e
R=${1:-r3}
H=$(git rev-parse --short HEAD)
for W in syn4x200_s1 PF08184 kinase syn8x400_s5; do
  python tools/pmc_summary.py gpurun_out/prof_$W $W --round $R --commit $H \
    --cmd "python3 bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-north-star --no-sub-records (syn8x400_s5: --steps 5 --warmup 2)" | tail -4
  cp gpurun_out/ev/bench_$W.json profiles/${R}_bench_$W.json
done
cp gpurun_out/ev/tests.log profiles/${R}_gpu_tests.log
cp gpurun_out/ev/sharded_one_gpu.txt profiles/${R}_sharded_one_gpu.txt
cp gpurun_out/ev/sharded_one_gpu_shift18.txt profiles/${R}_sharded_one_gpu_shift18.txt
cp gpurun_out/ev/many_probe.txt profiles/${R}_many_probe.txt
[ -f gpurun_out/ev/partial_probe.txt ] && cp gpurun_out/ev/partial_probe.txt profiles/${R}_partial_probe.txt
[ -f gpurun_out/ev/dive_phases.txt ] && cp gpurun_out/ev/dive_phases.txt profiles/${R}_dive_phases.txt
echo collected at $H
