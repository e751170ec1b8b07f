# Round 4: the sharded seen-set spill and merge-probe tests, the k_claim
# library A/B (LDS slot / bucket bits), the solo/narrow per-level costs, and
# the cold merge-probe A/B on NP=2 under a 4 GiB seen-set.
#   gpurun -- bash tools/gpu_r04_j.sh <tag>
set -o pipefail
TAG=${1:-r04j}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step spill_tests
timeout -k 10 700 python -u -m pytest tests/test_gpu_shard_seenspill.py tests/test_gpu_seenspill.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/spill_tests.log 2>&1 || { echo SPILL_TESTS_FAIL; tail -40 $O/spill_tests.log; exit 1; }
tail -3 $O/spill_tests.log
grep "NP=2" $O/spill_tests.log
step ablate
KC_ABLATE=1 timeout -k 10 300 python -u tools/exp_run.py --np 2 --runs 2 > $O/ablate.log 2>&1 || { echo ABLATE_FAIL; tail -20 $O/ablate.log; exit 1; }
grep "ablate" $O/ablate.log
step ab
L=tla-kubernetes_amd/kubecheck/lib
bash tools/gpu_r03_ab_lib.sh ${TAG}_ab $L/libkubecheck.so $L/libkubecheck_ldsmix.so $L/libkubecheck_bucketlow.so || exit 1
step levels
timeout -k 10 300 python -u tools/shard_levels.py --np2 > $O/shard_levels.log 2>&1 || { echo LEVELS_FAIL; tail -30 $O/shard_levels.log; exit 1; }
tail -2 $O/shard_levels.log
step redo
timeout -k 10 300 python -u tools/redo_cost.py > $O/redo_cost.log 2>&1 || { echo REDO_FAIL; tail -20 $O/redo_cost.log; exit 1; }
tail -1 $O/redo_cost.log
step merge_ab
for div in 0 16; do
  PYTHONPATH=$R/tla-kubernetes_amd KC_COLD_MERGE_DIV=$div timeout -k 10 200 python -u -c "
from kubecheck import ModelChecker, ModelConfig
import sys
with ModelChecker(ModelConfig(np=2, keep_trace=False, seen_hbm_bytes=4 << 30, verbose=1)) as mc:
    r = mc.run()
print('MERGE_DIV=$div', round(r.seconds, 3), r.distinct, r.seen)
" > $O/merge_$div.log 2>&1 || { echo MERGE_FAIL; tail -20 $O/merge_$div.log; exit 1; }
  grep -E "MERGE_DIV|seen-set spill" $O/merge_$div.log
done
step done
