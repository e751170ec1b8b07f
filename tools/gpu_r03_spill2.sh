# Seen-set spill: tests + the NP=2 4 GiB timing breakdown.
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== spill tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_seenspill.py -x -v -s --timeout 400 --timeout-method thread > $O/spill_tests.log 2>&1 || { echo SPILL_FAIL; tail -60 $O/spill_tests.log; exit 1; }
grep -E "PASS|FAIL|seen-set 4 GiB" $O/spill_tests.log
for V in "KC_SPILL_SYNC=0" "KC_SPILL_SYNC=1"; do
  echo "== spill np2 4 GiB, $V $(date +%T)"
  env $V timeout -k 10 300 python -u tools/spill_np2.py 4 > $O/spill_np2_4g_ab.json 2> $O/spill_np2_4g_ab.err || { echo SPILL_FAIL; tail -20 $O/spill_np2_4g_ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/spill_np2_4g_ab.json'));print(d['seconds'], d['exact'], d['seen'])"; grep "seen-set spill" $O/spill_np2_4g_ab.err
done
echo "== done $(date +%T)"
