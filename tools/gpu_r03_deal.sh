# k_claim dealt successor loop: engine GPU tests with the new library, the
# loop-occupancy diagnostic, and a same-box A/B against the lane = parent build.
set -o pipefail
TAG=${1:-r03ag}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
L=tla-kubernetes_amd/kubecheck/lib
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS_FAIL rc=$?"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
echo "== diag $(date +%T)"
KUBECHECK_LIB=$R/$L/libkubecheck_diag.so KC_ABLATE=1 timeout -k 10 300 python -u tools/exp_run.py --np 2 --runs 1 > $O/diagloop.log 2>&1 || { echo DIAG_FAIL; tail -20 $O/diagloop.log; exit 1; }
grep -v amdgpu.ids $O/diagloop.log
bash tools/gpu_r03_ab_lib.sh $TAG $L/libkubecheck.so $L/libkubecheck_nodeal.so
