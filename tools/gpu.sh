# GPU-box entry points (round 5: the one-off tools/gpu_r0*_*.sh scripts of
# rounds 3-4 folded into these subcommands; git history keeps the originals
# the round-3/4 profiles name).  Every GPU step runs under its own timeout and
# the steps are chained so that a failure ends the call.
#
#   gpurun -- bash tools/gpu.sh tests  <tag> [pytest args...]   GPU tests (default: all of -m gpu)
#   gpurun -- bash tools/gpu.sh round  <tag>                    tests, smoke, bench lines, NP=2 / FPSet
#                                                               traces + FETCH_SIZE / WRITE_SIZE passes
#                                                               (tools/gpu_round.sh), then part B below
#   gpurun -- bash tools/gpu.sh partb  <tag>                    NP=3 52-level trace + PMC + bench, the
#                                                               sharded k_claim PMC, the sharded bench
#                                                               line at world 1, per-level costs
#   gpurun -- bash tools/gpu.sh ab-lib <tag> <lib.so>...        same-box NP=2 benches of library builds
#   gpurun -- bash tools/gpu.sh ab-env <tag> "VAR=a" "-" ...    same-box NP=2 benches of env settings
#   gpurun -- bash tools/gpu.sh ab-fpset <tag> "VAR=a" "-" ...  same-box FPSet stress per env setting
#   gpurun -- bash tools/gpu.sh attr   <tag> [R...]             per-rank kernel attribution of the
#                                                               emulated sharded check (tools/gpu_attr.sh)
#   gpurun -- bash tools/gpu.sh levels <tag>                    per-level costs (tools/shard_levels.py --np2)
#   gpurun -- bash tools/gpu.sh probe  <tag>                    host probe: JVM / tla2tools.jar, CPUs
set -o pipefail
CMD=$1
TAG=${2:-x}
shift 2
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
B="python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
case "$CMD" in
tests)
  ARGS=${@:-tests -m gpu}
  step tests
  timeout -k 10 1000 python -u -m pytest $ARGS -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo TESTS_FAIL; grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
  ;;
round)
  bash tools/gpu_round.sh $TAG || exit 1
  cp $O/summary.json $R/profiles/${TAG}_np2_rocprof_summary.json
  cp $O/fpset_summary.json $R/profiles/${TAG}_fpset_rocprof_summary.json
  step bench_np2_pmc
  timeout -k 10 600 python -u bench.py > $O/bench_np2_pmc.json 2> $O/bench_np2_pmc.err \
    || { echo BENCH2_FAIL; tail -20 $O/bench_np2_pmc.err; exit 1; }
  cat $O/bench_np2_pmc.json
  bash tools/gpu.sh partb $TAG || exit 1
  ;;
partb)
  bash tools/gpu_r04_fin_b.sh $TAG || exit 1
  ;;
ab-lib)
  for rep in 1 2; do
    for L in "$@"; do
      n=$(basename $L .so)
      step "$n $rep"
      KUBECHECK_LIB=$R/$L timeout -k 10 300 $B > $O/${n}_$rep.json 2> $O/${n}_$rep.err \
        || { echo B_FAIL; tail -20 $O/${n}_$rep.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/${n}_$rep.json'));print(d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'])"
    done
  done
  ;;
ab-env)
  i=0
  for rep in 1 2; do
    for v in "$@"; do
      i=$((i+1))
      step "[$v] $rep"
      if [ "$v" = "-" ]; then E=""; else E="$v"; fi
      env $E timeout -k 10 300 $B > $O/run_$i.json 2> $O/run_$i.err || { echo B_FAIL; tail -20 $O/run_$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/run_$i.json'));print(d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'])"
    done
  done
  ;;
ab-fpset)
  # same-box FPSet stress (1e10 inserts + lookups) per env setting, 50% and 75% load
  i=0
  for load in 0.5 0.75; do
    for v in "$@"; do
      i=$((i+1))
      step "[$v] load $load"
      if [ "$v" = "-" ]; then E=""; else E="$v"; fi
      env $E timeout -k 10 400 python -u bench.py --workload fpset --fp-load $load --steps 2 --warmup 1 --no-cpu-baseline \
        > $O/fpset_$i.json 2> $O/fpset_$i.err || { echo F_FAIL; tail -20 $O/fpset_$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/fpset_$i.json'));c=d['config'];print(d['value'], c['inserts_per_s'], c['lookups_per_s'])"
    done
  done
  ;;
attr)
  bash tools/gpu_attr.sh $TAG "$@" || exit 1
  ;;
levels)
  step levels
  timeout -k 10 400 python -u tools/shard_levels.py --np2 > $O/shard_levels.log 2>&1 \
    || { echo LEVELS_FAIL; tail -30 $O/shard_levels.log; exit 1; }
  cat $O/shard_levels.log
  ;;
probe)
  {
    echo "command -v java:"; command -v java || echo "  (none)"
    echo "JAVA_HOME=${JAVA_HOME:-unset}"
    echo "ls /usr/lib/jvm:"; ls /usr/lib/jvm 2>&1 || true
    echo "find / -xdev -name 'tla2tools*.jar' (timeout 120 s):"
    timeout 120 find / -xdev -name 'tla2tools*.jar' 2>/dev/null || true
    nproc; grep -m1 "model name" /proc/cpuinfo; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"
  } > $O/probe.log 2>&1
  cat $O/probe.log
  ;;
*)
  sed -n 2,20p tools/gpu.sh
  exit 2
  ;;
esac
step done
