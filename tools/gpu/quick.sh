# GPU tests (optionally -k filtered) and one bench line of a workload (one gpurun call)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t_quick.log 2>&1 || { echo tests_fail; tail -60 gpurun_out/t_quick.log; exit 1; }
tail -3 gpurun_out/t_quick.log
timeout -k 10 300 python bench.py --workload ${WL:-PF08184} --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_quick.json 2> gpurun_out/b_quick.err || { echo bench_fail; tail gpurun_out/b_quick.err; exit 1; }
cat gpurun_out/b_quick.json
