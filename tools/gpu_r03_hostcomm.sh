# The one-shard-per-process native loop over gloo (tests/test_gpu_hostcomm.py)
# plus the shard tests as a regression check.
set -o pipefail
TAG=${1:-r03m}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
echo "== hostcomm $(date +%T)"
timeout -k 10 600 $PT tests/test_gpu_hostcomm.py > $O/hostcomm.log 2>&1 || { echo "HC_FAIL rc=$?"; tail -80 $O/hostcomm.log; exit 1; }
tail -3 $O/hostcomm.log
echo "== shard $(date +%T)"
timeout -k 10 600 $PT tests/test_gpu_shard.py > $O/shard.log 2>&1 || { echo "SH_FAIL rc=$?"; tail -60 $O/shard.log; exit 1; }
tail -3 $O/shard.log
echo "== done $(date +%T)"
