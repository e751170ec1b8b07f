# A/B: k_claim with the group's CASes issued back to back (KC_CLAIM_PIPE=1;
# batch 2 and 3) against the default, NP=2 bench lines (golden-checked).
#   gpurun -- bash tools/gpu_r04_pipe.sh <tag>
set -o pipefail
TAG=${1:-r04p}
R=$GRAFT_REPO_ROOT
cd $R
L=tla-kubernetes_amd/kubecheck/lib
bash tools/gpu_r03_ab_lib.sh ${TAG}_ab $L/libkubecheck.so $L/libkubecheck_pipe.so $L/libkubecheck_pipe3.so || exit 1
bash tools/gpu_r03_ab_lib.sh ${TAG}_ab2 $L/libkubecheck_pipe.so $L/libkubecheck.so || exit 1
