# Round-3 iteration: seen-set spill tests, then the sharded loop's per-level
# cost (tools/shard_levels.py).
#   gpurun -- bash tools/gpu_spill.sh <tag>
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== spill tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_seenspill.py -x -v -s --timeout 400 --timeout-method thread > $O/spill_tests.log 2>&1 || { echo SPILL_FAIL; tail -60 $O/spill_tests.log; exit 1; }
grep -E "PASS|FAIL|seen-set 4 GiB" $O/spill_tests.log
echo "== shard levels $(date +%T)"
timeout -k 10 600 python -u tools/shard_levels.py --np2 > $O/shard_levels.json 2> $O/shard_levels.err || { echo LEVELS_FAIL; tail -20 $O/shard_levels.err; exit 1; }
cat $O/shard_levels.json
echo "== done $(date +%T)"
