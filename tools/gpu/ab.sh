# A/B timing of the default workload: bench.py lines (ms per step) for the
# working tree, repeated; usage: bash tools/gpu/ab.sh [workload] [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
W=${1:-syn4x200_s1}; R=${2:-3}
for i in $(seq 1 $R); do
  timeout -k 10 120 python bench.py --workload $W --steps 50 --warmup 5 --no-cpu-baseline --no-north-star > gpurun_out/ab_$i.json 2>gpurun_out/ab_$i.err || { echo ab_fail; tail gpurun_out/ab_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$i.json').read().strip().splitlines()[-1]); print('ms/step %.3f loop %.3f exp %d launch %.1f us' % (d['ms_per_step'], d['search_loop_s']*1e3, d['expansions_per_search'], d['roofline']['avg_launch_us']))"
done
if [ -f tools/gpu/libpastar_gpu_old.so ]; then
  cp mpi_pastar_msa_amd/libpastar_gpu.so /tmp/new.so && cp tools/gpu/libpastar_gpu_old.so mpi_pastar_msa_amd/libpastar_gpu.so
  echo old:
  for i in $(seq 1 $R); do
    timeout -k 10 120 python bench.py --workload $W --steps 50 --warmup 5 --no-cpu-baseline --no-north-star > gpurun_out/abo_$i.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abo_$i.json').read().strip().splitlines()[-1]); print('ms/step %.3f loop %.3f exp %d launch %.1f us' % (d['ms_per_step'], d['search_loop_s']*1e3, d['expansions_per_search'], d['roofline']['avg_launch_us']))"
  done
  cp /tmp/new.so mpi_pastar_msa_amd/libpastar_gpu.so
fi
