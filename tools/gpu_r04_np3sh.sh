# Round 4: NP=3 (47 levels) through the sharded loop (4 emulated ranks).
#   gpurun -- bash tools/gpu_r04_np3sh.sh <tag>
set -o pipefail
TAG=${1:-r04q}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_shard.py -k "np3_47 or enlarged_full" -x -v -s --durations=0 --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -8 $O/tests.log
