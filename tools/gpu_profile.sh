# rocprofv3 passes over one bench step (NP=2 model): kernel trace + stats,
# then FETCH_SIZE and WRITE_SIZE in separate PMC passes (MI355X_MICROARCH.md
# §HBM / rocprofv3 PMC slots: FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2).
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline"
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/trace -o run -- $BENCH > $R/gpurun_out/prof/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $R/gpurun_out/prof/trace.log; exit 1; }
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/fetch -o run -- $BENCH > $R/gpurun_out/prof/fetch.log 2>&1 || { echo FETCH_FAIL; tail -20 $R/gpurun_out/prof/fetch.log; exit 1; }
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/write -o run -- $BENCH > $R/gpurun_out/prof/write.log 2>&1 || { echo WRITE_FAIL; tail -20 $R/gpurun_out/prof/write.log; exit 1; }
find $R/gpurun_out/prof -name "*.csv" | head -20
