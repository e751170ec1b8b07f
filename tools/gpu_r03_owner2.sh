# New owner projection: every GPU test, the records each emulated rank count
# sends (new vs previous library), and the NP=2 bench A/B.
set -o pipefail
TAG=${1:-r03ac}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
L=tla-kubernetes_amd/kubecheck/lib
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS_FAIL rc=$?"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
echo "== records new $(date +%T)"
timeout -k 10 400 python -u tools/shard_records.py 2 4 8 > $O/records_new.log 2>&1 || { echo REC_FAIL; tail -20 $O/records_new.log; exit 1; }
grep '^{' $O/records_new.log
echo "== records prev $(date +%T)"
KUBECHECK_LIB=$R/$L/libkubecheck_prev.so timeout -k 10 400 python -u tools/shard_records.py 2 4 8 > $O/records_prev.log 2>&1 || { echo RECP_FAIL; tail -20 $O/records_prev.log; exit 1; }
grep '^{' $O/records_prev.log
bash tools/gpu_r03_ab_lib.sh $TAG $L/libkubecheck.so $L/libkubecheck_prev.so
