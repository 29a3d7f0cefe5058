cd $GRAFT_REPO_ROOT
export PASTAR_TIMING_MASK=1
for t in 17 18 20 22 24; do
echo "== table 2^$t"
TABLE_LOG2=$t timeout -k 10 300 python tools/gpu/probe.py syn4x200_s1,PF08184 3 0 2>&1 | grep -v "step [0-9]* expanded"
done
for p in 65536 1048576 16777216; do
echo "== pool $p"
POOL=$p TABLE_LOG2=20 timeout -k 10 300 python tools/gpu/probe.py syn4x200_s1 3 0 2>&1 | grep -v "step [0-9]* expanded"
done
