# Sharded path after the round-3 changes: per-level cost (tools/shard_levels.py:
# engine, RCCL world 1, emulated ranks) and the bench --sharded line at world 1.
set -o pipefail
TAG=${1:-r03at}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== shard_levels $(date +%T)"
timeout -k 10 600 python -u tools/shard_levels.py --np2 > $O/shard_levels.log 2>&1 || { echo SL_FAIL; tail -30 $O/shard_levels.log; exit 1; }
grep -v amdgpu.ids $O/shard_levels.log | tail -20
bash tools/gpu_r03_sharded_bench.sh $TAG
