# Round 5: the narrow-level changes: GPU tests of the engine and the sharded
# loop, the Model_1 narrow phase trace (KC_NARROW_TRACE=1), per-level costs.
#   gpurun -- bash tools/gpu_r05_narrow.sh <tag>
set -o pipefail
TAG=${1:-r05q}
R0=$GRAFT_REPO_ROOT
cd $R0
O=$R0/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_shard.py tests/test_gpu_hostcomm.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
KC_NARROW_TRACE=1 timeout -k 10 200 python -u -c "
import sys, time; sys.path.insert(0, 'tla-kubernetes_amd')
import torch
from kubecheck import ModelChecker, ModelConfig
mc = ModelChecker(ModelConfig())
for k in range(3):
    t = time.perf_counter(); r = mc.run(); print('check', k, round((time.perf_counter() - t) * 1e3, 3), 'ms', r.distinct, r.depth, flush=True)
" > $O/ntrace.log 2>&1 || { echo NTRACE_FAIL; tail -20 $O/ntrace.log; exit 1; }
tail -2 $O/ntrace.log
timeout -k 10 400 python -u tools/shard_levels.py --np2 > $O/shard_levels.log 2>&1 || { echo LEVELS_FAIL; tail -30 $O/shard_levels.log; exit 1; }
grep '^{' $O/shard_levels.log
