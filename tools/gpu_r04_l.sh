# Round 4: the sharded tests with the split narrow emit, per-level costs and
# a kernel trace of the narrow levels at world 1.
#   gpurun -- bash tools/gpu_r04_l.sh <tag>
set -o pipefail
TAG=${1:-r04l}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step shard_tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_hostcomm.py tests/test_gpu_shard_seenspill.py -x -q --timeout 200 --timeout-method thread > $O/shard_tests.log 2>&1 || { echo SHARD_TESTS_FAIL; tail -40 $O/shard_tests.log; exit 1; }
tail -2 $O/shard_tests.log
step levels
timeout -k 10 300 python -u tools/shard_levels.py > $O/shard_levels.log 2>&1 || { echo LEVELS_FAIL; tail -30 $O/shard_levels.log; exit 1; }
tail -1 $O/shard_levels.log
step sn_trace
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sntrace -o run -- python3 $R/tools/sn_trace.py --force > $O/sntrace.log 2>&1 || { echo SNTRACE_FAIL; tail -20 $O/sntrace.log; exit 1; }
cd $R
find $O/sntrace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/sn_kernel_stats.csv
head -5 $O/sn_kernel_stats.csv | cut -c1-60,200-
step done
