# k_claim / k_emit ablation times (KC_ABLATE=1, product library; the ablated
# run takes the materialising path)
set -o pipefail
TAG=${1:-r03z}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
KC_ABLATE=1 timeout -k 10 300 python -u tools/exp_run.py --np 2 --runs 2 > $O/ablate.log 2>&1 || { echo ABL_FAIL; tail -20 $O/ablate.log; exit 1; }
grep -v amdgpu.ids $O/ablate.log
