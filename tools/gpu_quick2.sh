# quick GPU iteration: engine tests + Model_1/NP=2 bench lines.
#   gpurun -- bash tools/gpu_quick2.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-q}
K=${2:-}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
if [ -n "$K" ]; then KARG="-k $K"; else KARG=""; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread $KARG > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -50 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "== model1 $(date +%T)"
timeout -k 10 300 python -u bench.py --workload model1 --steps 10 --warmup 2 --no-cpu-baseline > $O/model1.json 2> $O/model1.err || { echo M1_FAIL; tail -20 $O/model1.err; exit 1; }
cat $O/model1.json
echo "== np2 $(date +%T)"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/np2.json 2> $O/np2.err || { echo NP2_FAIL; tail -20 $O/np2.err; exit 1; }
cat $O/np2.json
