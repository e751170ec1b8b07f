# Round-3 iteration: host-link microbench + seen-set spill tests + the native
# sharded loop's tests.
#   gpurun -- bash tools/gpu_spill.sh <tag>
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== host_probe $(date +%T)"
timeout -k 10 240 ./tools/microbench/host_probe > $O/host_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/host_probe.txt; exit 1; }
cat $O/host_probe.txt
echo "== engine tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_tlc_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/engine_tests.log 2>&1 || { echo ENGINE_FAIL; tail -60 $O/engine_tests.log; exit 1; }
tail -3 $O/engine_tests.log
echo "== shard tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -v -k "native" --timeout 300 --timeout-method thread > $O/shard_tests.log 2>&1 || { echo SHARD_FAIL; tail -60 $O/shard_tests.log; exit 1; }
tail -5 $O/shard_tests.log
echo "== spill tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_seenspill.py -x -v -s --timeout 600 --timeout-method thread > $O/spill_tests.log 2>&1 || { echo SPILL_FAIL; tail -60 $O/spill_tests.log; exit 1; }
tail -30 $O/spill_tests.log
echo "== done $(date +%T)"
