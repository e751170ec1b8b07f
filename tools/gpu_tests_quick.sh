# Run the given GPU test files.   gpurun -- bash tools/gpu_tests_quick.sh <tag> <files...>
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
