# Round 4: sharded tests, level costs, the k_claim A/B of the locate /
# fingerprint variants, then the NP=3 52-level golden (host CPUs) and its
# GPU check and bench line.
#   gpurun -- bash tools/gpu_r04_g.sh <tag>
set -o pipefail
TAG=${1:-r04g}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step shard_tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_hostcomm.py -x -v --timeout 200 --timeout-method thread > $O/shard_tests.log 2>&1 || { echo SHARD_TESTS_FAIL; tail -60 $O/shard_tests.log; exit 1; }
tail -2 $O/shard_tests.log
step levels
timeout -k 10 300 python -u tools/shard_levels.py --np2 > $O/shard_levels.log 2>&1 || { echo LEVELS_FAIL; tail -30 $O/shard_levels.log; exit 1; }
tail -2 $O/shard_levels.log
L=tla-kubernetes_amd/kubecheck/lib
bash tools/gpu_r03_ab_lib.sh ${TAG}_ab $L/libkubecheck.so $L/libkubecheck_swar.so $L/libkubecheck_fold.so $L/libkubecheck_both.so || exit 1
step np3_golden
( bash tools/np3_golden.sh $O/np3_52levels.json > $O/np3_golden.log 2>&1 ) &
P=$!
while kill -0 $P 2>/dev/null; do sleep 30; echo "  np3 golden running $(date +%T)"; done
wait $P || { echo GOLDEN_FAIL; tail $O/np3_golden.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/np3_52levels.json')); print({k: d[k] for k in ('distinct','generated','depth','seconds','set_full')})"
cp $O/np3_52levels.json tests/golden/np3_52levels.json
step np3_test
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -k np3 -x -v --timeout 240 --timeout-method thread > $O/np3_test.log 2>&1 || { echo NP3_TEST_FAIL; tail -40 $O/np3_test.log; exit 1; }
tail -2 $O/np3_test.log
step np3_bench
timeout -k 10 400 python -u bench.py --workload np3_52 --steps 3 --warmup 1 --cpu-seconds 10 > $O/bench_np3.json 2> $O/bench_np3.err || { echo NP3_BENCH_FAIL; tail -20 $O/bench_np3.err; exit 1; }
cat $O/bench_np3.json
step done
