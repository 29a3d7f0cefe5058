# depth x depth_full grid on N = 5, 6 inputs (tools/gpu/depth_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
for F in ${FULLS:-4 6 8}; do
  echo "depth_full=$F"
  PASTAR_DEPTH_FULL=$F timeout -k 10 600 python tools/gpu/depth_probe.py "${DEPTHS:-8,12,16,32}" 3 $@ || exit 1
done
