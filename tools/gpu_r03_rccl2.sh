# Probe: two RCCL ranks (two processes) on one GPU through the native
# sharded loop (tools/rccl_two_ranks_one_gpu.py).
set -o pipefail
TAG=${1:-r03l}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp NCCL_DEBUG=WARN
echo "== rccl2 model1 $(date +%T)"
timeout -k 10 180 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
  --master-port=29577 tools/rccl_two_ranks_one_gpu.py --trace > $O/rccl2.log 2>&1 || { echo "RCCL2_FAIL rc=$?"; tail -40 $O/rccl2.log; exit 1; }
grep '^{' $O/rccl2.log
echo "== rccl2 np2 $(date +%T)"
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
  --master-port=29578 tools/rccl_two_ranks_one_gpu.py --np2 > $O/rccl2_np2.log 2>&1 || { echo "RCCL2NP2_FAIL rc=$?"; tail -40 $O/rccl2_np2.log; exit 1; }
grep '^{' $O/rccl2_np2.log
echo "== done $(date +%T)"
