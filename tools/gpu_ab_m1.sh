# Same-box A/B of Model_1 (bench.py --workload model1) under environment
# settings, alternating, after the engine GPU tests.
#   gpurun -- bash tools/gpu_ab_m1.sh <tag> "ENV=VAL" "ENV=VAL" ...
set -o pipefail
TAG=$1
shift
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for round in 1 2 3; do
  k=0
  for e in "$@"; do
    k=$((k+1))
    env $e timeout -k 10 300 python -u bench.py --workload model1 --steps 30 --warmup 3 --no-cpu-baseline > $O/m1_${k}_$round.json 2> $O/m1_${k}_$round.err || { echo M1_FAIL; tail -20 $O/m1_${k}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/m1_${k}_$round.json')); print('[$e]', $round, d['ms_per_step'])"
  done
done
