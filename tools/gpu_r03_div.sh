# Divergence study (tools/divergence_study.py) on captured NP=2 levels.
set -o pipefail
TAG=${1:-r03ao}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u tools/divergence_study.py 50 86 120 > $O/div.log 2>&1 || { echo DIV_FAIL; tail -20 $O/div.log; exit 1; }
grep '^{' $O/div.log
