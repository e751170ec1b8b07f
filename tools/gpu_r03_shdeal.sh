# Sharded k_claim with the deal: shard GPU tests, then emulated R = 2/4/8
# whole-NP=2 checks with and without the deal (same box, twice).
set -o pipefail
TAG=${1:-r03aq}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
L=tla-kubernetes_amd/kubecheck/lib
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_hostcomm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS_FAIL rc=$?"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for rep in 1 2; do
  :
  for lib in libkubecheck libkubecheck_nodeal; do
    echo "== $lib $rep $(date +%T)"
    KUBECHECK_LIB=$R/$L/$lib.so timeout -k 10 400 python -u tools/shard_records.py 2 4 8 > $O/${lib}_$rep.log 2>&1 || { echo REC_FAIL; tail -20 $O/${lib}_$rep.log; exit 1; }
    grep '^{' $O/${lib}_$rep.log | python3 -c "import sys,json;[print(d['R'],d['ms'],d['distinct']) for d in map(json.loads,sys.stdin)]"
  done
done
bash tools/gpu_r03_env_ab.sh $TAG KC_CS_CLEAR=memset - KC_CS_CLEAR=kernel:16384
