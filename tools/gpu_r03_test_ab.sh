# Engine GPU tests on the default library, then a same-box A/B of builds.
#   gpurun -- bash tools/gpu_r03_test_ab.sh <tag> <lib1> <lib2> ...
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== engine tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py > $O/engine.log 2>&1 || { echo "ENG_FAIL rc=$?"; tail -60 $O/engine.log; exit 1; }
tail -2 $O/engine.log
bash tools/gpu_r03_ab_lib.sh "$@"
