# Round-2 GPU call: parity tests, smoke, bench lines (NP=2 default, Model_1,
# FPSet stress).  gpurun -- bash tools/gpu_r02.sh <tag> [tests|bench|all]
set -o pipefail
TAG=${1:-r02}
WHAT=${2:-all}
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/$TAG
O=$R/gpurun_out/$TAG
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
step bench_np2
timeout -k 10 600 python -u bench.py > $O/bench_np2.json 2> $O/bench_np2.err || { echo BENCH2_FAIL; tail -20 $O/bench_np2.err; exit 1; }
cat $O/bench_np2.json
step bench_model1
timeout -k 10 300 python -u bench.py --workload model1 --steps 5 --warmup 1 --cpu-seconds 5 > $O/bench_model1.json 2> $O/bench_model1.err || { echo BENCH1_FAIL; tail -20 $O/bench_model1.err; exit 1; }
cat $O/bench_model1.json
step bench_fpset
timeout -k 10 300 python -u bench.py --workload fpset --steps 2 --warmup 1 > $O/bench_fpset.json 2> $O/bench_fpset.err || { echo BENCHF_FAIL; tail -20 $O/bench_fpset.err; exit 1; }
cat $O/bench_fpset.json
fi
step done
