# sharded-path GPU checks: shard tests (emulated ranks, RCCL world 1) and the
# sharded bench line at world 1 (native C++ level loop; Python loop beside it)
set -o pipefail
TAG=${1:-s}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== shard tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "== sharded bench native world 1 $(date +%T)"
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533 bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline > $O/sharded_native.json 2> $O/sharded_native.err || { echo SN_FAIL; tail -30 $O/sharded_native.err; exit 1; }
cat $O/sharded_native.json
echo "== sharded bench python world 1 $(date +%T)"
KC_PY_DRIVER=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29534 bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline > $O/sharded_py.json 2> $O/sharded_py.err || { echo SP_FAIL; tail -30 $O/sharded_py.err; exit 1; }
cat $O/sharded_py.json
