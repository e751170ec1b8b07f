# ClaimSet 32 vs 64 GiB on the whole NP=2 model (deferred frontier), twice each.
set -o pipefail
TAG=${1:-r03s}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/locality_ab.py --full-only > $O/locality.log 2>&1 || { echo "LOC_FAIL rc=$?"; tail -30 $O/locality.log; exit 1; }
grep '^{' $O/locality.log
