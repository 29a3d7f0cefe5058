# rocprofv3 kernel trace + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of
# bench.py on a workload.  Usage: bash tools/gpu/profile_round1.sh WORKLOAD [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
W=$1; shift
OUT=gpurun_out/prof_$W
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --workload $W --no-cpu-baseline "$@" > $OUT/bench_trace.json 2> $OUT/trace.err || { echo trace_fail; tail -20 $OUT/trace.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- \
    python3 bench.py --workload $W --no-cpu-baseline "$@" > $OUT/bench_fetch.json 2> $OUT/fetch.err || { echo fetch_fail; tail -20 $OUT/fetch.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- \
    python3 bench.py --workload $W --no-cpu-baseline "$@" > $OUT/bench_write.json 2> $OUT/write.err || { echo write_fail; tail -20 $OUT/write.err; exit 1; }
find $OUT -name '*.csv' | head -20
