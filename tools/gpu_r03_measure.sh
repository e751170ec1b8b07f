# Round-3 measurements: seen-set spill breakdown (NP=2 at 4 GiB, host and
# disk tiers), NP=3 sizing, kc_fpset_put from T threads.
#   gpurun -- bash tools/gpu_r03_measure.sh <tag>
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== spill np2 4 GiB $(date +%T)"
timeout -k 10 300 python -u tools/spill_np2.py 4 > $O/spill_np2_4g.json 2> $O/spill_np2_4g.err || { echo SPILL_FAIL; tail -20 $O/spill_np2_4g.err; exit 1; }
cat $O/spill_np2_4g.json; grep "seen-set spill" $O/spill_np2_4g.err
for V in "KC_COLD_CACHE=0" "KC_SEEN_HOT_DIV=4" "KC_SEEN_HOT_DIV=4 KC_COLD_BLOOM_BITS=6" "KC_SPILL_SYNC=1"; do
  echo "== spill np2 4 GiB, $V $(date +%T)"
  env $V timeout -k 10 300 python -u tools/spill_np2.py 4 > $O/spill_np2_4g_ab.json 2> $O/spill_np2_4g_ab.err || { echo SPILL_FAIL; tail -20 $O/spill_np2_4g_ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/spill_np2_4g_ab.json'));print(d['seconds'], d['exact'], d['seen'])"; grep "seen-set spill" $O/spill_np2_4g_ab.err
done
echo "== np3 sizing $(date +%T)"
timeout -k 10 300 python -u tools/np3_size.py 45 50 > $O/np3_size.json 2> $O/np3_size.err || { echo NP3_FAIL; tail -20 $O/np3_size.err; exit 1; }
cut -c1-400 $O/np3_size.json
echo "== fpset put threads $(date +%T)"
timeout -k 10 120 ./tools/microbench/fpset_put_threads 2 > $O/fpset_put_threads.json 2>&1 || { echo PUT_FAIL; tail -20 $O/fpset_put_threads.json; exit 1; }
cat $O/fpset_put_threads.json
echo "== done $(date +%T)"
