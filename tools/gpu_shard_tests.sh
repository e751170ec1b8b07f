# The sharded GPU tests (emulated ranks, RCCL world 1, one shard per process
# over gloo, seen-set spill per rank), then the attribution of R = 8.
#   gpurun -- bash tools/gpu_shard_tests.sh <tag> [R ...]
set -o pipefail
TAG=${1:-shard}
shift
R0=$GRAFT_REPO_ROOT
O=$R0/gpurun_out/$TAG
mkdir -p $O
cd $R0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${KC_TESTS:-tests/test_gpu_shard.py tests/test_gpu_hostcomm.py tests/test_gpu_shard_seenspill.py} > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|error" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
[ -n "$1" ] && bash tools/gpu_attr.sh $TAG/attr "$@"
exit 0
