# Spare ClaimSet cleared on a side stream: engine GPU tests, then the NP=2
# bench with and without it (KC_CS_SPARE=0), same box.
set -o pipefail
TAG=${1:-r03ai}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS_FAIL rc=$?"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/gpu_r03_env_ab.sh $TAG - KC_CS_SPARE=0
