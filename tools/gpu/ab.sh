# A/B timing: the working tree's library against tools/gpu/libpastar_gpu_old.so,
# alternating processes; usage: bash tools/gpu/ab.sh [workload] [pairs] [steps]
set -o pipefail
cd $GRAFT_REPO_ROOT
W=${1:-syn4x200_s1}; R=${2:-4}; S=${3:-100}
cp mpi_pastar_msa_amd/libpastar_gpu.so /tmp/new.so
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2 ms/step %.3f loop %.3f exp %d launch %.1f us' % (d['ms_per_step'], d['search_loop_s']*1e3, d['expansions_per_search'], d['roofline']['avg_launch_us']))"; }
for i in $(seq 1 $R); do
  for v in new old; do
    if [ $v = old ]; then cp ${OLD_SO:-tools/gpu/libpastar_gpu_old.so} mpi_pastar_msa_amd/libpastar_gpu.so; else cp /tmp/new.so mpi_pastar_msa_amd/libpastar_gpu.so; fi
    timeout -k 10 120 python bench.py --workload $W --steps $S --warmup 5 --no-cpu-baseline --no-north-star $AB_ARGS > gpurun_out/ab_$v$i.json 2>gpurun_out/ab_$v$i.err || { echo ab_fail; tail gpurun_out/ab_$v$i.err; cp /tmp/new.so mpi_pastar_msa_amd/libpastar_gpu.so; exit 1; }
    line gpurun_out/ab_$v$i.json $v
  done
done
cp /tmp/new.so mpi_pastar_msa_amd/libpastar_gpu.so
