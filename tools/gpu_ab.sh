# Same-box A/B of engine switches: the NP=2 check under each environment
# setting in turn (tools/exp_run.py, per-kernel HIP events, 3 runs each),
# twice round, after the engine parity tests with the switches on.
#   gpurun -- bash tools/gpu_ab.sh <tag> "ENV=VAL ENV2=VAL" "ENV=VAL" ...
set -o pipefail
TAG=${1:-ab}
shift
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
echo "== tests (all switches on) $(date +%T)"
env $1 timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_squeue.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for round in 1 2; do
  k=0
  for e in "$@"; do
    k=$((k+1))
    echo "== [$e] round $round $(date +%T)"
    env $e timeout -k 10 300 python -u tools/exp_run.py --runs 3 > $O/exp_${k}_$round.log 2>&1 || { echo EXP_FAIL; tail -20 $O/exp_${k}_$round.log; exit 1; }
    grep "^run [12]" $O/exp_${k}_$round.log
  done
done
