# A/B of the per-action counter stripes (libkubecheck_s1 = one stripe), then
# the full round (tools/gpu_round.sh) on the product library.
set -o pipefail
TAG=${1:-r03as}
R=$GRAFT_REPO_ROOT
cd $R
L=tla-kubernetes_amd/kubecheck/lib
bash tools/gpu_r03_ab_lib.sh ${TAG}_ab $L/libkubecheck.so $L/libkubecheck_s1.so || exit 1
bash tools/gpu_round.sh $TAG
