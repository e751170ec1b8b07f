# One GPU iteration: engine parity tests, the KC_DIAG ablation run, then the
# NP=2 and Model_1 bench lines of the product library.
#   gpurun -- bash tools/gpu_iter.sh <tag> [pytest files...]
set -o pipefail
TAG=${1:-iter}
shift
T=${@:-tests/test_gpu_engine.py tests/test_gpu_squeue.py}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "== diag $(date +%T)"
KUBECHECK_LIB=$R/tla-kubernetes_amd/kubecheck/lib/libkubecheck_diag.so KC_ABLATE=1 timeout -k 10 300 python -u tools/exp_run.py --runs 2 > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -20 $O/diag.log; exit 1; }
grep -v amdgpu.ids $O/diag.log
echo "== np2 $(date +%T)"
timeout -k 10 300 python -u tools/exp_run.py --runs 3 > $O/exp_run.log 2>&1 || { echo EXP_FAIL; tail -20 $O/exp_run.log; exit 1; }
grep -v amdgpu.ids $O/exp_run.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/np2.json 2> $O/np2.err || { echo NP2_FAIL; tail -20 $O/np2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/np2.json')); print('np2', d['ms_per_step'], d['value'], d['kernel_ms_per_step'], d['roofline']['frac'])"
echo "== model1 $(date +%T)"
timeout -k 10 300 python -u bench.py --workload model1 --steps 10 --warmup 2 --no-cpu-baseline > $O/model1.json 2> $O/model1.err || { echo M1_FAIL; tail -20 $O/model1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/model1.json')); print('model1', d['ms_per_step'], d['value'], d['kernel_ms_per_step'])"
