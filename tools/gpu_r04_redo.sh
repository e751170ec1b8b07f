# Engine redo-from-level tests + sharded tests + level costs.
#   gpurun -- bash tools/gpu_r04_redo.sh <tag>
set -o pipefail
TAG=${1:-r04e}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step engine_tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread > $O/engine_tests.log 2>&1 || { echo ENGINE_TESTS_FAIL; tail -60 $O/engine_tests.log; exit 1; }
tail -3 $O/engine_tests.log
step shard_tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_hostcomm.py -x -v --timeout 200 --timeout-method thread > $O/shard_tests.log 2>&1 || { echo SHARD_TESTS_FAIL; tail -60 $O/shard_tests.log; exit 1; }
tail -3 $O/shard_tests.log
step levels
timeout -k 10 300 python -u tools/shard_levels.py > $O/shard_levels.log 2>&1 || { echo LEVELS_FAIL; tail -30 $O/shard_levels.log; exit 1; }
tail -1 $O/shard_levels.log
step done
