# Diagnostic run: the KC_DIAG library with KC_ABLATE=1 (k_claim outcome
# counters, cut-down k_claim / k_emit variants), then the product bench.
#   gpurun -- bash tools/gpu_diag.sh <tag> [np]
set -o pipefail
TAG=${1:-diag}
NP=${2:-2}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
echo "== diag $(date +%T)"
KUBECHECK_LIB=$R/tla-kubernetes_amd/kubecheck/lib/libkubecheck_diag.so KC_ABLATE=1 timeout -k 10 300 python -u tools/exp_run.py --np $NP --runs 2 > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -20 $O/diag.log; exit 1; }
grep -v amdgpu.ids $O/diag.log
echo "== bench $(date +%T)"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/np2.json 2> $O/np2.err || { echo NP2_FAIL; tail -20 $O/np2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/np2.json')); print(d['ms_per_step'], d['value'], d['kernel_ms_per_step'], d['roofline']['frac'])"
