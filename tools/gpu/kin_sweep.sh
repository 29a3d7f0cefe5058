# kinase / syn8x400 continuation-policy sweep (PASTAR_DEEP_ROUNDS)
set -o pipefail
cd $GRAFT_REPO_ROOT
for R in ${ROUNDS:-16 8 4 2}; do
  echo "== deep_rounds $R"
  PASTAR_DEEP_ROUNDS=$R timeout -k 10 200 python tools/gpu/probe.py ${WL:-kinase} 3 || exit 1
done
