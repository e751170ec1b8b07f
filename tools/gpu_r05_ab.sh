# Round 5 A/Bs in one call: engine tests with 4 tiles per settle workgroup,
# the NP=2 bench at 1/2/4/8 tiles per settle workgroup, the FPSet stress
# with and without windowed inserts, and the sharded loop's per-level costs.
#   gpurun -- bash tools/gpu_r05_ab.sh <tag>
set -o pipefail
TAG=${1:-r05e}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
KC_SETTLE_TP=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $O/engine_tests_tp4.log 2>&1 || { echo ENGINE_TESTS_FAIL; tail -30 $O/engine_tests_tp4.log; exit 1; }
tail -2 $O/engine_tests_tp4.log
bash tools/gpu.sh ab-env ${TAG}/settle "-" "KC_SETTLE_TP=2" "KC_SETTLE_TP=4" "KC_SETTLE_TP=8" || exit 1
bash tools/gpu.sh ab-fpset ${TAG}/fpset "-" "KC_STRESS_WINDOW=27" "KC_STRESS_WINDOW=25" || exit 1
bash tools/gpu.sh levels ${TAG}/levels || exit 1
