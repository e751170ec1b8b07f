# The N-GPU bench path at world 1 (bench.py --sharded self-launches under
# torch.distributed.run; native loop over RCCL), NP=2 and the sharded FPSet.
set -o pipefail
TAG=${1:-r03aa}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== sharded np2 $(date +%T)"
timeout -k 10 400 python -u bench.py --sharded --steps 3 --warmup 1 > $O/sh_np2.json 2> $O/sh_np2.err || { echo SH_FAIL; tail -30 $O/sh_np2.err; exit 1; }
cat $O/sh_np2.json
echo "== sharded fpset $(date +%T)"
timeout -k 10 400 python -u bench.py --sharded --workload fpset --steps 1 --warmup 1 > $O/sh_fpset.json 2> $O/sh_fpset.err || { echo SHF_FAIL; tail -30 $O/sh_fpset.err; exit 1; }
cat $O/sh_fpset.json
echo "== done $(date +%T)"
