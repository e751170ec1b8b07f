# k_claim successor-loop occupancy (KC_DIAG build): wave trips vs lane trips,
# and the trips if each tile's parents were dealt to waves by successor count
set -o pipefail
TAG=${1:-r03af}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
KUBECHECK_LIB=$R/tla-kubernetes_amd/kubecheck/lib/libkubecheck_diag.so KC_ABLATE=1 timeout -k 10 300 python -u tools/exp_run.py --np 2 --runs 1 > $O/diagloop.log 2>&1 || { echo DIAG_FAIL; tail -20 $O/diagloop.log; exit 1; }
grep -v amdgpu.ids $O/diagloop.log
