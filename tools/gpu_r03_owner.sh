# Owner-function study (tools/owner_balance.py) on captured NP=2 levels.
set -o pipefail
TAG=${1:-r03ab}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u tools/owner_balance.py > $O/owner.log 2>&1 || { echo OWN_FAIL; tail -20 $O/owner.log; exit 1; }
grep '^{' $O/owner.log
