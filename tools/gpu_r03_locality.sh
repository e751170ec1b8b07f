# Locality A/B (tools/locality_ab.py): k_claim time vs ClaimSet size for the same work.
set -o pipefail
TAG=${1:-r03n}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== locality $(date +%T)"
timeout -k 10 600 python -u tools/locality_ab.py > $O/locality.log 2>&1 || { echo "LOC_FAIL rc=$?"; tail -30 $O/locality.log; exit 1; }
grep '^{' $O/locality.log
echo "== done $(date +%T)"
