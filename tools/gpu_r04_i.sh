# A/B of the LDS slot hash (libkubecheck_ldsmix = rounds 1-3's remixed slot),
# then the round-4 GPU round (tools/gpu_r04_round.sh).
#   gpurun -- bash tools/gpu_r04_i.sh <tag>
set -o pipefail
TAG=${1:-r04i}
R=$GRAFT_REPO_ROOT
cd $R
L=tla-kubernetes_amd/kubecheck/lib
bash tools/gpu_r03_ab_lib.sh ${TAG}_ab $L/libkubecheck.so $L/libkubecheck_ldsmix.so $L/libkubecheck_bucketlow.so || exit 1
bash tools/gpu_r04_round.sh $TAG
