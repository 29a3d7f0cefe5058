# Where the expand kernel's wave cycles go: issue (ACTIVE_INST_ANY), parked
# on s_waitcnt / barriers (WAIT_ANY) or issue stalls (WAIT_INST_ANY), with
# the instruction mix, per workload.  Two --pmc passes per workload (8 SQ
# counters each), kernel trace only.
#   bash tools/gpu/pmc_stalls.sh syn4x200_s1 kinase
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/stalls
mkdir -p $out
for W in "$@"; do
  args="--workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-north-star"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU \
    -d $out/${W}_a -o p --output-format csv -- python3 bench.py $args > $out/${W}_a.log 2>&1 || { echo pass_a_fail $W; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH \
    -d $out/${W}_b -o p --output-format csv -- python3 bench.py $args > $out/${W}_b.log 2>&1 || { echo pass_b_fail $W; exit 1; }
done
echo stalls_ok
