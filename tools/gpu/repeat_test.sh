# one GPU test repeated in fresh processes until it fails (its report is kept)
# or the count is reached; usage: bash tools/gpu/repeat_test.sh "<pytest -k expression>" [count]
cd $GRAFT_REPO_ROOT
K=$1; N=${2:-30}
for i in $(seq 1 $N); do
  timeout -k 10 100 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 90 --timeout-method thread -k "$K" > gpurun_out/rep.log 2>&1 || { echo "failed at run $i"; grep -E "^E  |assert|Error" gpurun_out/rep.log | head -20; exit 0; }
done
echo "$N runs passed"
