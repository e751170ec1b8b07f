# Deferred frontier A/B on one box: plans passed between levels (default),
# KC_DEFER_PC=0 (rebuilds plan their grandparent), KC_DEFER=0 (materialising).
set -o pipefail
TAG=${1:-r03r}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
echo "== engine tests $(date +%T)"
timeout -k 10 600 $PT tests/test_gpu_engine.py > $O/engine.log 2>&1 || { echo "ENG_FAIL rc=$?"; tail -60 $O/engine.log; exit 1; }
tail -2 $O/engine.log
B="python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
for rep in 1 2; do
for v in "KC_DEFER=1" "KC_DEFER_PC=0" "KC_DEFER=0"; do
  echo "== bench np2 $v $(date +%T)"
  env $v timeout -k 10 300 $B > $O/np2_${v}_$rep.json 2> $O/np2_${v}_$rep.err || { echo "B_FAIL"; tail -20 $O/np2_${v}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/np2_${v}_$rep.json'));print(d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'])"
done
done
echo "== done $(date +%T)"
