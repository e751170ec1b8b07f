# Round 4 GPU round: every GPU test, smoke, the bench lines and profiles of
# NP=2 (rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes), the NP=3
# 52-level workload and the FPSet stress (tools/gpu_round.sh), then the
# sharded per-level costs.
#   gpurun -- bash tools/gpu_r04_round.sh <tag>
set -o pipefail
TAG=${1:-r04h}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
bash tools/gpu_round.sh $TAG || exit 1
step() { echo "== $1 $(date +%T)"; }
step bench_np3
timeout -k 10 400 python -u bench.py --workload np3_52 --steps 3 --warmup 1 --cpu-seconds 10 > $O/bench_np3.json 2> $O/bench_np3.err || { echo NP3_BENCH_FAIL; tail -20 $O/bench_np3.err; exit 1; }
cat $O/bench_np3.json
BENCH="$R/bench.py --workload np3_52 --steps 1 --warmup 1 --no-cpu-baseline --no-timing"
cd /tmp
step np3_trace
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n3trace -o run -- python3 $BENCH > $O/n3trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/n3trace.log; exit 1; }
cd $R
python3 tools/pmc_summary.py --trace $O/n3trace --out $O/np3_summary.json --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --workload np3_52 --steps 1 --warmup 1 --no-cpu-baseline --no-timing"
step levels
timeout -k 10 300 python -u tools/shard_levels.py --np2 > $O/shard_levels.log 2>&1 || { echo LEVELS_FAIL; tail -30 $O/shard_levels.log; exit 1; }
tail -2 $O/shard_levels.log
step done
