# rocprofv3 kernel trace of Model_1 bench steps (per-kernel durations and gaps)
set -o pipefail
TAG=${1:-t}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --workload model1 --steps 3 --warmup 1 --no-cpu-baseline --no-timing > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs cat | head -20
