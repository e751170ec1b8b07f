# Round 4: the added sharded seen-set spill parity tests (NP=2 lost update,
# NP=2 40-level prefix, emulated and one shard per process over gloo), the
# engine tests with the direct report of deferred invariant violations, and
# the time to a counterexample (tools/redo_cost.py).
#   gpurun -- bash tools/gpu_r04_m.sh <tag>
set -o pipefail
TAG=${1:-r04m}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $O/engine_tests.log 2>&1 || { echo ENGINE_TESTS_FAIL; tail -40 $O/engine_tests.log; exit 1; }
tail -2 $O/engine_tests.log
timeout -k 10 300 python -u tools/redo_cost.py > $O/redo_cost.log 2>&1 || { echo REDO_FAIL; tail -20 $O/redo_cost.log; exit 1; }
tail -1 $O/redo_cost.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_seenspill.py tests/test_gpu_hostcomm.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
