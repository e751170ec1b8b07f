# Sharded paths at world 1 on one GPU (RCCL world 1 through torch.distributed.run):
# the owner-sharded FPSet stress (BASELINE config 4) and the native C++ sharded
# BFS level loop, beside the single-GPU engine on the same box.
#   gpurun -- bash tools/gpu_shard_r02.sh <tag>
set -o pipefail
TAG=${1:-sh}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
echo "== fpset sharded $(date +%T)"
timeout -k 10 400 $TR --master-port 29511 bench.py --workload fpset --sharded --steps 1 --warmup 1 > $O/fpset_sharded.json 2> $O/fpset_sharded.err || { echo FPS_FAIL; tail -30 $O/fpset_sharded.err; exit 1; }
cat $O/fpset_sharded.json
echo "== np2 sharded $(date +%T)"
timeout -k 10 300 $TR --master-port 29512 bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline > $O/np2_sharded.json 2> $O/np2_sharded.err || { echo NP2S_FAIL; tail -30 $O/np2_sharded.err; exit 1; }
cat $O/np2_sharded.json
echo "== np2 engine $(date +%T)"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/np2.json 2> $O/np2.err || { echo NP2_FAIL; tail -30 $O/np2.err; exit 1; }
cat $O/np2.json
echo "== done $(date +%T)"
