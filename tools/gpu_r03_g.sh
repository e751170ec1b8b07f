# Round 3 check after the overflow-settle fold: engine + spill + squeue +
# fpset tests, the put microbench, then the np2 / model1 bench lines.
set -o pipefail
TAG=${1:-r03g}
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
run engine 600 $PT tests/test_gpu_engine.py
run spill 600 $PT tests/test_gpu_seenspill.py tests/test_gpu_squeue.py
run fpset 300 $PT tests/test_gpu_fpset.py
run put 120 ./tools/microbench/fpset_put_threads 2
cat $O/put.log
run bench_np2 300 python bench.py
run bench_m1 300 python bench.py --workload model1
echo "== done $(date +%T)"
