# Round 4: engine tests (device parent-chain walk), the one-multiply
# fingerprint mix A/B (NP=2 bench, NP=3 52-level golden), redo cost, the
# cold check's synchronous time with and without the merge-probe, and a
# kernel trace of the sharded narrow levels at world 1.
#   gpurun -- bash tools/gpu_r04_k.sh <tag>
set -o pipefail
TAG=${1:-r04k}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
L=tla-kubernetes_amd/kubecheck/lib
step() { echo "== $1 $(date +%T)"; }
step engine_tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $O/engine_tests.log 2>&1 || { echo ENGINE_TESTS_FAIL; tail -40 $O/engine_tests.log; exit 1; }
tail -2 $O/engine_tests.log
step redo
timeout -k 10 300 python -u tools/redo_cost.py > $O/redo_cost.log 2>&1 || { echo REDO_FAIL; tail -20 $O/redo_cost.log; exit 1; }
tail -1 $O/redo_cost.log
step ab
bash tools/gpu_r03_ab_lib.sh ${TAG}_ab $L/libkubecheck.so $L/libkubecheck_mix1.so || exit 1
step np3_mix1
KUBECHECK_LIB=$R/$L/libkubecheck_mix1.so timeout -k 10 400 python -u bench.py --workload np3_52 --steps 1 --warmup 1 --no-cpu-baseline > $O/np3_mix1.json 2> $O/np3_mix1.err || { echo NP3_MIX1_FAIL; tail -20 $O/np3_mix1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/np3_mix1.json'));print(d['ms_per_step'], d['config'].get('golden_check'))"
step spill_sync
for div in 0 16; do
  PYTHONPATH=$R/tla-kubernetes_amd KC_SPILL_SYNC=1 KC_COLD_MERGE_DIV=$div timeout -k 10 200 python -u -c "
from kubecheck import ModelChecker, ModelConfig
with ModelChecker(ModelConfig(np=2, keep_trace=False, seen_hbm_bytes=4 << 30, verbose=1)) as mc:
    r = mc.run()
print('MERGE_DIV=$div', round(r.seconds, 3), r.distinct, r.seen)
" > $O/spill_sync_$div.log 2>&1 || { echo SPILL_FAIL; tail -20 $O/spill_sync_$div.log; exit 1; }
  grep -E "MERGE_DIV|seen-set spill" $O/spill_sync_$div.log
done
step sn_trace
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sntrace -o run -- python3 $R/tools/sn_trace.py --force > $O/sntrace.log 2>&1 || { echo SNTRACE_FAIL; tail -20 $O/sntrace.log; exit 1; }
cd $R
find $O/sntrace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/sn_kernel_stats.csv
head -12 $O/sn_kernel_stats.csv
step done
