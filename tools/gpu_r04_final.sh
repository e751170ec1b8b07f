# Round 4 final GPU round in one call: tools/gpu_round.sh (every GPU test,
# smoke, bench lines, NP=2 and FPSet traces + FETCH_SIZE / WRITE_SIZE passes),
# the NP=2 bench line again with this build's PMC in the box's profiles/, then
# tools/gpu_r04_fin_b.sh (NP=3 52 levels, sharded k_claim PMC, sharded bench,
# per-level costs).
#   gpurun -- bash tools/gpu_r04_final.sh <tag>
set -o pipefail
TAG=${1:-r04y}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
bash tools/gpu_round.sh $TAG || exit 1
cp $O/summary.json $R/profiles/${TAG}_np2_rocprof_summary.json
cp $O/fpset_summary.json $R/profiles/${TAG}_fpset_rocprof_summary.json
echo "== bench_np2_pmc $(date +%T)"
timeout -k 10 600 python -u bench.py > $O/bench_np2_pmc.json 2> $O/bench_np2_pmc.err || { echo BENCH2_FAIL; tail -20 $O/bench_np2_pmc.err; exit 1; }
cat $O/bench_np2_pmc.json
bash tools/gpu_r04_fin_b.sh $TAG || exit 1
