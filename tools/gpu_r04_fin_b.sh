# Round 4 final, part B (part A: tools/gpu_round.sh): the NP=3 52-level bench
# with its kernel trace and FETCH_SIZE / WRITE_SIZE passes, the sharded
# k_claim's PMC (NP=2, 8 emulated ranks), the sharded bench line at world 1,
# and the sharded loop's per-level costs.
#   gpurun -- bash tools/gpu_r04_fin_b.sh <tag>
set -o pipefail
TAG=${1:-r04x}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
B3="$R/bench.py --workload np3_52 --steps 1 --warmup 1 --no-cpu-baseline --no-timing"
cd /tmp
step np3_trace
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n3trace -o run -- python3 $B3 > $O/n3trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/n3trace.log; exit 1; }
step np3_fetch
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/n3fetch -o run -- python3 $B3 > $O/n3fetch.log 2>&1 || { echo FETCH_FAIL; tail -20 $O/n3fetch.log; exit 1; }
step np3_write
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/n3write -o run -- python3 $B3 > $O/n3write.log 2>&1 || { echo WRITE_FAIL; tail -20 $O/n3write.log; exit 1; }
cd $R
python3 tools/pmc_summary.py --trace $O/n3trace --fetch $O/n3fetch --write $O/n3write --out $O/np3_summary.json --command "rocprofv3 -- python3 bench.py --workload np3_52 --steps 1 --warmup 1 --no-cpu-baseline --no-timing"
# (the box's copy of profiles/: the bench lines below find this build's PMC)
cp $O/np3_summary.json $R/profiles/${TAG}_np3_52_rocprof_summary.json
step bench_np3
timeout -k 10 400 python -u bench.py --workload np3_52 --steps 3 --warmup 1 --cpu-seconds 10 > $O/bench_np3.json 2> $O/bench_np3.err || { echo NP3_BENCH_FAIL; tail -20 $O/bench_np3.err; exit 1; }
cat $O/bench_np3.json
step sharded_pmc
timeout -k 10 120 python -u tools/sharded_profile.py 8 --out $O/sh_alg.json || { echo ALG_FAIL; exit 1; }
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shtrace -o run -- python3 $R/tools/sharded_profile.py 8 > $O/shtrace.log 2>&1 || { echo SHTRACE_FAIL; tail -20 $O/shtrace.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/shfetch -o run -- python3 $R/tools/sharded_profile.py 8 > $O/shfetch.log 2>&1 || { echo SHFETCH_FAIL; tail -20 $O/shfetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/shwrite -o run -- python3 $R/tools/sharded_profile.py 8 > $O/shwrite.log 2>&1 || { echo SHWRITE_FAIL; tail -20 $O/shwrite.log; exit 1; }
cd $R
python3 tools/pmc_summary.py --trace $O/shtrace --fetch $O/shfetch --write $O/shwrite --algorithmic $O/sh_alg.json --out $O/np2_sharded_summary.json --command "rocprofv3 -- python3 tools/sharded_profile.py 8 (NP=2, 8 ranks emulated on one GPU)"
cp $O/np2_sharded_summary.json $R/profiles/${TAG}_np2_sharded_rocprof_summary.json
step bench_sharded
timeout -k 10 400 python -u bench.py --sharded --steps 3 --warmup 1 --cpu-seconds 10 > $O/bench_np2_sharded_world1.json 2> $O/bench_sharded.err || { echo SHBENCH_FAIL; tail -20 $O/bench_sharded.err; exit 1; }
cat $O/bench_np2_sharded_world1.json
step levels
timeout -k 10 300 python -u tools/shard_levels.py --np2 > $O/shard_levels.log 2>&1 || { echo LEVELS_FAIL; tail -30 $O/shard_levels.log; exit 1; }
tail -2 $O/shard_levels.log
step done
