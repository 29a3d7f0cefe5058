cd $GRAFT_REPO_ROOT
for m in 7 1; do
echo "== mask $m"
PASTAR_TIMING_MASK=$m timeout -k 10 300 python tools/gpu/probe.py syn4x200_s1,PF08184,kinase,syn8x400_s5 3 0 v 2>&1 | grep -v "step [0-9]* expanded"
done
