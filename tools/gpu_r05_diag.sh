# Round 5: error reports per switch (tools/diag_errors.py) at R = 1, 2, 3.
set -o pipefail
TAG=${1:-r05diag}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/diag_errors.py 1 2 3 > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag.log; exit 1; }
grep '^{' $O/diag.log
