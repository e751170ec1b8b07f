# Engine tests (redo from the anomaly's level), sharded tests and per-level
# costs (narrow levels fused), then the k_claim A/B (tools/gpu_r03_ab_lib.sh)
# of the locate / fingerprint variants.
#   gpurun -- bash tools/gpu_r04_f.sh <tag>
set -o pipefail
TAG=${1:-r04f}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_r04_redo.sh $TAG || exit 1
L=tla-kubernetes_amd/kubecheck/lib
bash tools/gpu_r03_ab_lib.sh ${TAG}_ab $L/libkubecheck.so $L/libkubecheck_swar.so $L/libkubecheck_fold.so $L/libkubecheck_both.so
