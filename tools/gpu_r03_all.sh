# Round-3 call: the new GPU tests, then the measurements and the sharded PMC profile.
#   gpurun -- bash tools/gpu_r03_all.sh <tag>
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_squeue.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash tools/gpu_r03_measure.sh $TAG || exit 1
bash tools/gpu_r03_shprof.sh $TAG || exit 1
echo "== random probe vs table size $(date +%T)"
timeout -k 10 300 ./tools/microbench/random_probe > $O/random_probe.txt 2>&1 || { echo RP_FAIL; tail -5 $O/random_probe.txt; exit 1; }
cat $O/random_probe.txt
echo "== all done $(date +%T)"
