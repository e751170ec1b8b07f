# Round 4: the sharded seen-set spill and hostcomm tests.
#   gpurun -- bash tools/gpu_r04_n.sh <tag>
set -o pipefail
TAG=${1:-r04n}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_seenspill.py tests/test_gpu_hostcomm.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
