# full GPU test suite, smoke, default bench, then rocprofv3 trace + PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout=400 > gpurun_out/t_all.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || { echo smoke_fail; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/b_default.json 2> gpurun_out/b_default.err || { echo bench_fail; tail gpurun_out/b_default.err; exit 1; }
cat gpurun_out/b_default.json
for W in syn4x200_s1 kinase syn8x400_s5; do
  OUT=gpurun_out/prof_$W; mkdir -p $OUT
  EXTRA=""; [ $W = syn8x400_s5 ] && EXTRA="--table-log2 28"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline $EXTRA > $OUT/bench.json 2> $OUT/trace.err || { echo trace_fail $W; tail $OUT/trace.err; exit 1; }
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline $EXTRA > /dev/null 2> $OUT/fetch.err || { echo fetch_fail $W; tail $OUT/fetch.err; exit 1; }
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline $EXTRA > /dev/null 2> $OUT/write.err || { echo write_fail $W; tail $OUT/write.err; exit 1; }
  cat $OUT/bench.json
done
