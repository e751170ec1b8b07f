# One GPU call: parity tests, smoke, bench lines (Model_1, NP=2), a rocprofv3
# kernel trace of one NP=2 bench step and FETCH_SIZE / WRITE_SIZE PMC passes
# (separate runs: MI355X_MICROARCH.md rocprofv3 PMC slots).
#   gpurun -- bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/$TAG
O=$R/gpurun_out/$TAG
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
step bench_model1
timeout -k 10 300 python -u bench.py --workload model1 --steps 5 --warmup 1 --cpu-seconds 5 > $O/bench_model1.json 2> $O/bench_model1.err || { echo BENCH1_FAIL; tail -20 $O/bench_model1.err; exit 1; }
cat $O/bench_model1.json
step bench_np2
timeout -k 10 600 python -u bench.py > $O/bench_np2.json 2> $O/bench_np2.err || { echo BENCH2_FAIL; tail -20 $O/bench_np2.err; exit 1; }
cat $O/bench_np2.json
BENCH="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-timing"
cd /tmp
step trace
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $BENCH > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.log; exit 1; }
step fetch
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $BENCH > $O/fetch.log 2>&1 || { echo FETCH_FAIL; tail -20 $O/fetch.log; exit 1; }
step write
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $BENCH > $O/write.log 2>&1 || { echo WRITE_FAIL; tail -20 $O/write.log; exit 1; }
cd $R
python3 tools/pmc_summary.py --trace $O/trace --fetch $O/fetch --write $O/write --out $O/summary.json --command "rocprofv3 -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-timing"
# FPSet stress (BASELINE config 4): the bench line at 1e10 fps, PMC passes at 2^30
step bench_fpset
timeout -k 10 300 python -u bench.py --workload fpset --steps 2 --warmup 1 > $O/bench_fpset.json 2> $O/bench_fpset.err || { echo BENCHF_FAIL; tail -20 $O/bench_fpset.err; exit 1; }
cat $O/bench_fpset.json
FBENCH="$R/bench.py --workload fpset --fp-count 1073741824 --steps 1 --warmup 0"
cd /tmp
step fpset_trace
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ftrace -o run -- python3 $FBENCH > $O/ftrace.log 2>&1 || { echo FTRACE_FAIL; tail -20 $O/ftrace.log; exit 1; }
step fpset_fetch
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/ffetch -o run -- python3 $FBENCH > $O/ffetch.log 2>&1 || { echo FFETCH_FAIL; tail -20 $O/ffetch.log; exit 1; }
step fpset_write
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/fwrite -o run -- python3 $FBENCH > $O/fwrite.log 2>&1 || { echo FWRITE_FAIL; tail -20 $O/fwrite.log; exit 1; }
cd $R
python3 tools/pmc_summary.py --trace $O/ftrace --fetch $O/ffetch --write $O/fwrite --out $O/fpset_summary.json --command "rocprofv3 -- python3 bench.py --workload fpset --fp-count 1073741824 --steps 1 --warmup 0"
step done
