set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --cpu-seconds 3 > gpurun_out/b_default.json 2> gpurun_out/b_default.err || { echo bench_fail; tail gpurun_out/b_default.err; exit 1; }
cat gpurun_out/b_default.json
timeout -k 10 300 python bench.py --workload kinase --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_kin.json 2>&1; tail -c 600 gpurun_out/b_kin.json
echo; echo "--- 2 ranks on one GPU (RCCL may refuse a duplicate GPU)"
PASTAR_BENCH_DEVICE=0 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/b_2r.log 2>&1; echo rc=$?; tail -5 gpurun_out/b_2r.log
