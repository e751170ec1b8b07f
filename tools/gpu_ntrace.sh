# Narrow-level phase timestamps (KC_NARROW_TRACE=1) for Model_1 and the
# Model_1 bench line.   gpurun -- bash tools/gpu_ntrace.sh <tag>
set -o pipefail
TAG=${1:-ntrace}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
KC_NARROW_TRACE=1 timeout -k 10 300 python -u tools/exp_run.py --np 1 --runs 3 > $O/ntrace.log 2>&1 || { echo NT_FAIL; tail -20 $O/ntrace.log; exit 1; }
grep -v amdgpu.ids $O/ntrace.log | tail -8
timeout -k 10 300 python -u bench.py --workload model1 --steps 20 --warmup 3 --no-cpu-baseline > $O/model1.json 2> $O/model1.err || { echo M1_FAIL; tail -20 $O/model1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/model1.json')); print('model1', d['ms_per_step'], d['kernel_ms_per_step'])"
if [ "$2" = diag ]; then
  KUBECHECK_LIB=$R/tla-kubernetes_amd/kubecheck/lib/libkubecheck_diag.so KC_ABLATE=1 timeout -k 10 300 python -u tools/exp_run.py --runs 2 > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -20 $O/diag.log; exit 1; }
  grep -v amdgpu.ids $O/diag.log | tail -4
fi
