# Shard-path iteration 2: shard parity tests, then the native sharded NP=2
# bench at world 1 with RCCL forced, device-row gather (default) vs host
# rows (KC_DEVROW=0), alternating.   gpurun -- bash tools/gpu_shard_iter2.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for round in 1 2; do
  for v in 1 0; do
    KC_DEVROW=$v KC_RCCL_FORCE=1 timeout -k 10 300 python -u bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline > $O/shf_${v}_$round.json 2> $O/shf_${v}_$round.err || { echo SHF_FAIL; tail -20 $O/shf_${v}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/shf_${v}_$round.json')); print('devrow=$v RCCL forced', d['ms_per_step'], d['config'].get('golden_check'))"
  done
done
