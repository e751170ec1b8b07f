# A/B: settle pass B with the overflow list in the same launch
# (KC_SETTLE_FUSE=1) against the default; the engine and seen-set spill tests
# on the variant first.
#   gpurun -- bash tools/gpu_r04_fuse.sh <tag>
set -o pipefail
TAG=${1:-r04f2}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
L=tla-kubernetes_amd/kubecheck/lib
KUBECHECK_LIB=$R/$L/libkubecheck_fuse.so timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_seenspill.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_r03_ab_lib.sh ${TAG}_ab $L/libkubecheck.so $L/libkubecheck_fuse.so || exit 1
bash tools/gpu_r03_ab_lib.sh ${TAG}_ab2 $L/libkubecheck_fuse.so $L/libkubecheck.so || exit 1
