# The whole GPU test suite and smoke on the final tree.
#   gpurun -- bash tools/gpu_r04_tests.sh <tag>
set -o pipefail
TAG=${1:-r04t}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -20 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
