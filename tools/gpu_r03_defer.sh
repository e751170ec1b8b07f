# Deferred frontier: engine GPU tests, then NP=2 bench deferred vs KC_DEFER=0 on the same box.
set -o pipefail
TAG=${1:-r03o}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
echo "== engine tests $(date +%T)"
timeout -k 10 600 $PT tests/test_gpu_engine.py > $O/engine.log 2>&1 || { echo "ENG_FAIL rc=$?"; tail -60 $O/engine.log; exit 1; }
tail -3 $O/engine.log
B="python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
for k in 1 0 1 0; do
  echo "== bench np2 KC_DEFER=$k $(date +%T)"
  KC_DEFER=$k timeout -k 10 300 $B > $O/np2_d$k.json 2> $O/np2_d$k.err || { echo "B_FAIL"; tail -20 $O/np2_d$k.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/np2_d$k.json'));print(d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'])"
done
echo "== bench model1 $(date +%T)"
timeout -k 10 300 python -u bench.py --workload model1 --steps 5 --warmup 1 --no-cpu-baseline > $O/m1.json 2> $O/m1.err || { echo "M1_FAIL"; tail -20 $O/m1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/m1.json'));print(d['ms_per_step'])"
echo "== done $(date +%T)"
