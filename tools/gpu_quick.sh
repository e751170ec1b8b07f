# Quick GPU iteration: parity tests, then the NP=2 bench (no CPU baseline).
#   gpurun -- bash tools/gpu_quick.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-q}
shift
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/bench_np2.json 2> $O/bench_np2.err || { echo BENCH_FAIL; tail -20 $O/bench_np2.err; exit 1; }
cat $O/bench_np2.json
