# every extra input (tools/tune_inputs, the small golden ones in batched mode)
# under several builds of the library; usage: bash tools/gpu/inputs_ab.sh "tag1 tag2"
cd $GRAFT_REPO_ROOT
cp mpi_pastar_msa_amd/libpastar_gpu.so /tmp/keep.so
for f in tools/tune_inputs/*.fasta tests/golden/test2.fasta tests/golden/PF08184.fasta tests/golden/syn8x100_s3.fasta; do
  for t in $1; do
    cp tools/gpu/libpastar_gpu_$t.so mpi_pastar_msa_amd/libpastar_gpu.so
    TAG=$t timeout -k 10 120 python tools/gpu/file_probe.py $f 8 batched || { cp /tmp/keep.so mpi_pastar_msa_amd/libpastar_gpu.so; exit 1; }
  done
done
cp /tmp/keep.so mpi_pastar_msa_amd/libpastar_gpu.so
