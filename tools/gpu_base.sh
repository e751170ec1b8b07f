# Baseline breakdown of the current tree: per-kernel HIP-event times of the
# NP=2 check (tools/exp_run.py), then a rocprofv3 kernel trace of the bench.
#   gpurun -- bash tools/gpu_base.sh <tag>
set -o pipefail
TAG=${1:-base}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== exp_run $(date +%T)"
timeout -k 10 300 python -u tools/exp_run.py --runs 3 > $O/exp_run.log 2>&1 || { echo EXP_FAIL; tail -20 $O/exp_run.log; exit 1; }
cat $O/exp_run.log
echo "== trace $(date +%T)"
bash tools/gpu_prof_r02.sh $TAG np2 || exit 1
