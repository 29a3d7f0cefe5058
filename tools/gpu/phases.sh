# Expand-kernel diagnostics: block-0 phase timers and per-block chain
# statistics (tools/gpu/libpastar_gpu_phases.so, built with
# PASTAR_HIPCC_FLAGS=-DPASTAR_PHASE_TIMERS) on the given workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
cp mpi_pastar_msa_amd/libpastar_gpu.so /tmp/keep.so
cp tools/gpu/libpastar_gpu_phases.so mpi_pastar_msa_amd/libpastar_gpu.so
PASTAR_TIMING_MASK=5 timeout -k 10 150 python tools/gpu/engine_probe.py ${1:-syn4x200_s1,kinase} batched ${2:-3} > gpurun_out/phases.log 2>&1
rc=$?
cp /tmp/keep.so mpi_pastar_msa_amd/libpastar_gpu.so
grep -v "^\[pastar\] step" gpurun_out/phases.log
exit $rc
