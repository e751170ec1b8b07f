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
split)
  # the split claim (KC_SPLIT): engine tests with it on, then same-box NP=2 A/B
  step tests
  KC_SPLIT=4 timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "enlarged_full or first_claim or error_paths or deferred or model1" > $O/tests.log 2>&1 \
    || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
  bash tools/gpu.sh ab-env ${TAG}_ab - KC_SPLIT=2 KC_SPLIT=4 KC_SPLIT=8 || exit 1
  ;;
trace)
  # rocprofv3 kernel trace of one NP=2 bench check under the given env (e.g. KC_SPLIT=2)
  cd /tmp
  step trace
  env $3 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-first-claim-line > $O/trace.log 2>&1 \
    || { echo TRACE_FAIL; tail -20 $O/trace.log; exit 1; }
  cd $R
  f=$(ls $O/trace/*/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -12 "$f"
  ;;
graph)
  # the narrow batch as a hipGraph (KC_NARROW_GRAPH=1): Model_1 tests with it on, Model_1 A/B, the new NP=2 line
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/tests_all.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error" $O/tests_all.log | head; tail -30 $O/tests_all.log; exit 1; }
  tail -2 $O/tests_all.log
  KC_NARROW_GRAPH=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "model1 or error_paths or narrow" > $O/tests.log 2>&1 \
    || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
  i=0
  for rep in 1 2; do
    for v in - KC_NARROW_GRAPH=1; do
      i=$((i+1)); step "model1 [$v] $rep"
      if [ "$v" = "-" ]; then E=""; else E="$v"; fi
      env $E timeout -k 10 300 python -u bench.py --workload model1 --steps 20 --warmup 2 --no-cpu-baseline \
        > $O/m1_$i.json 2> $O/m1_$i.err || { echo M1_FAIL; tail -20 $O/m1_$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/m1_$i.json'));print(d['ms_per_step'], d.get('kernel_ms_per_step'))"
    done
  done
  step bench_np2
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_np2.json 2> $O/bench_np2.err \
    || { echo BENCH_FAIL; tail -20 $O/bench_np2.err; exit 1; }
  cat $O/bench_np2.json
  ;;
abtest)
  # tests under an env setting ($3), then same-box NP=2 benches: default vs $3 (twice each)
  step tests
  env $3 timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "${TESTK:-first_claim}" > $O/tests.log 2>&1 \
    || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
  bash tools/gpu.sh ab-env ${TAG}_ab - "$3" || exit 1
  ;;
power)
  # power and clocks sampled while NP=2 checks run (is k_claim power/clock-limited?)
  step idle
  timeout 20 rocm-smi --showpower --showclocks > $O/idle.txt 2>&1; grep -iE "power|sclk|mclk|fclk" $O/idle.txt | head -8
  step run
  ( for k in $(seq 1 60); do echo "== t $k"; timeout 5 rocm-smi --showpower --showclocks 2>&1 | grep -iE "power|sclk|mclk"; sleep 0.2; done ) > $O/busy.txt 2>&1 &
  SP=$!
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 1 --no-cpu-baseline --no-second-line > $O/bench.json 2> $O/bench.err \
    || { echo BENCH_FAIL; tail -20 $O/bench.err; kill $SP; exit 1; }
  wait $SP
  python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['ms_per_step'], d['kernel_ms_per_step'])"
  grep -iE "power|sclk" $O/busy.txt | sort | uniq -c | sort -rn | head -20
  ;;
abk)
  # same-box NP=2 A/B of env settings (args after the tag; "-" = none) with
  # HIP events on every kernel, headline mode only, REPS rounds
  shift 2
  i=0
  for rep in $(seq 1 ${REPS:-3}); do
    for v in "$@"; do
      i=$((i+1)); step "[$v] $rep"
      if [ "$v" = "-" ]; then E=""; else E="$v"; fi
      env $E timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 1 --no-cpu-baseline --no-second-line \
        --all-kernel-timing $BARGS > $O/run_$i.json 2> $O/run_$i.err || { echo B_FAIL; tail -20 $O/run_$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/run_$i.json'));print(d['ms_per_step'], {k: round(v, 2) for k, v in d['kernel_ms_per_step'].items()})"
    done
  done
  ;;
*)
  sed -n 1,8p tools/gpu_r06.sh
  exit 2
  ;;
esac
step done
