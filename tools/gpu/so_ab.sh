# bench.py lines of a workload under several builds of the library, alternating
# (tools/gpu/libpastar_gpu_<tag>.so); usage: bash tools/gpu/so_ab.sh "tag1 tag2 ..." [workload] [steps] [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAGS=$1; W=${2:-syn4x200_s1}; S=${3:-40}; R=${4:-2}
cp mpi_pastar_msa_amd/libpastar_gpu.so /tmp/keep.so
for i in $(seq 1 $R); do for t in $TAGS; do
  cp tools/gpu/libpastar_gpu_$t.so mpi_pastar_msa_amd/libpastar_gpu.so
  timeout -k 10 120 python bench.py --workload $W --steps $S --warmup 5 --no-cpu-baseline --no-north-star --no-sub-records > gpurun_out/sw.json 2>gpurun_out/sw.err || { echo fail $t; tail gpurun_out/sw.err; cp /tmp/keep.so mpi_pastar_msa_amd/libpastar_gpu.so; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('$t $W ms/step %.3f loop %.3f exp %d steps %.1f launch %.1f us ok %s' % (d['ms_per_step'], d['search_loop_s']*1e3, d['expansions_per_search'], d['steps_per_search'], d['roofline']['avg_launch_us'], d['score_ok']))"
done; done
cp /tmp/keep.so mpi_pastar_msa_amd/libpastar_gpu.so
