# FPSet seam: the GPU FPSet tests, then kc_fpset_put from 1/4/16/64 threads.
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== fpset tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fpset.py -x -v --timeout 300 --timeout-method thread > $O/fpset_tests.log 2>&1 || { echo TESTS_FAIL; tail -60 $O/fpset_tests.log; exit 1; }
tail -3 $O/fpset_tests.log
echo "== fpset put threads $(date +%T)"
timeout -k 10 120 ./tools/microbench/fpset_put_threads 2 > $O/fpset_put_threads.json 2>&1 || { echo PUT_FAIL; tail -20 $O/fpset_put_threads.json; exit 1; }
cat $O/fpset_put_threads.json
echo "== done $(date +%T)"
