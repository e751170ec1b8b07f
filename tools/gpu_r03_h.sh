# Sharded loop after the launch fusion: shard + gloo-free GPU shard tests,
# per-level cost (tools/shard_levels.py --np2), the put microbench.
set -o pipefail
TAG=${1:-r03h}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
run() {   # name seconds cmd...
  local n=$1 t=$2; shift 2
  echo "== $n $(date +%T)"
  timeout -k 10 $t "$@" > $O/$n.log 2>&1 || { echo "FAIL $n rc=$?"; tail -60 $O/$n.log; exit 1; }
  tail -3 $O/$n.log
}
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run shard 900 $PT tests/test_gpu_shard.py
run levels 600 python -u tools/shard_levels.py --np2
cat $O/levels.log
#run put 120 ./tools/microbench/fpset_put_threads 2
#cat $O/put.log
echo "== done $(date +%T)"
