# Engine parity tests, then the narrow trace and Model_1 bench (tools/gpu_ntrace.sh).
#   gpurun -- bash tools/gpu_nt2.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_squeue.py tests/test_gpu_shard.py tests/test_tlc_cli.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/$1/tests.log; exit 1; }
tail -1 gpurun_out/$1/tests.log
bash tools/gpu_ntrace.sh $1
