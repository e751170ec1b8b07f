# Same-box A/B of two libraries on the native sharded NP=2 path at world 1
# with RCCL forced, alternating; shard parity tests first.
#   gpurun -- bash tools/gpu_ab_shard2.sh <tag> <libB.so>
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for round in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export KUBECHECK_LIB=$R/tla-kubernetes_amd/kubecheck/lib/$2; else unset KUBECHECK_LIB; fi
    KC_RCCL_FORCE=1 timeout -k 10 300 python -u bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline > $O/s_${v}_$round.json 2> $O/s_${v}_$round.err || { echo BENCH_FAIL; tail -20 $O/s_${v}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s_${v}_$round.json')); print('$v', $round, d['ms_per_step'])"
  done
done
unset KUBECHECK_LIB
