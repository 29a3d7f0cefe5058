# rocprofv3 kernel-trace + separate FETCH_SIZE / WRITE_SIZE passes of bench.py
# for each workload, each under the command the driver runs for the default
# workload (--steps 20 --warmup 5; no CPU legs, no north-star record, which
# only add host time); the summaries into profiles/ are made on the CPU side
# (tools/pmc_summary.py).  Usage: bash tools/gpu/profile_all.sh W1 [W2 ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for W in "$@"; do
  OUT=gpurun_out/prof_$W; rm -rf $OUT; mkdir -p $OUT
  EXTRA=""
  STEPS="--steps 20 --warmup 5"; [ $W = syn8x400_s5 ] && STEPS="--steps 5 --warmup 2"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload $W $STEPS --no-cpu-baseline --no-north-star --no-sub-records $EXTRA > $OUT/bench.json 2> $OUT/trace.err || { echo trace_fail $W; tail $OUT/trace.err; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-north-star --no-sub-records $EXTRA > /dev/null 2> $OUT/fetch.err || { echo fetch_fail $W; tail $OUT/fetch.err; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-north-star --no-sub-records $EXTRA > /dev/null 2> $OUT/write.err || { echo write_fail $W; tail $OUT/write.err; exit 1; }
  cat $OUT/bench.json
done
