# Round-6 GPU steps (same conventions as tools/gpu.sh: every GPU step under
# its own timeout, the first failure ends the call).
#   gpurun -- bash tools/gpu_r06.sh first <tag>    ceiling microbench, first-claim GPU tests,
#                                                  NP=2 bench, emulated R=8 walls in both claim modes
set -o pipefail
CMD=$1
TAG=${2:-x}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
case "$CMD" in
first)
  if [ -z "$SKIP_CEIL" ]; then
    step ceiling
    timeout -k 10 240 ./tools/microbench/claim_ceiling > $O/ceiling.log 2>&1 || { echo CEIL_FAIL; tail $O/ceiling.log; exit 1; }
    tail -1 $O/ceiling.log
  fi
  step tests
  timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_engine.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "${TESTK:-first_claim or enlarged_full or counted_deferred or error_paths}" > $O/tests.log 2>&1 \
    || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
  step bench
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_np2.json 2> $O/bench_np2.err \
    || { echo BENCH_FAIL; tail $O/bench_np2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_np2.json'));print(d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'], d.get('first_claim'))"
  for M in "" "--first"; do
    step "R=8 $M"
    timeout -k 10 300 python -u tools/shard_attr.py run 8 --checks 3 $M > $O/wall_R8$M.log 2>&1 || { echo WALL_FAIL; tail -20 $O/wall_R8$M.log; exit 1; }
    grep '^{' $O/wall_R8$M.log | tail -2
  done
  ATTR_ARGS=--first bash tools/gpu.sh attr ${TAG}_attr 8 || exit 1
  ;;
*)
  sed -n 1,8p tools/gpu_r06.sh
  exit 2
  ;;
esac
step done
