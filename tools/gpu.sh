# GPU-box entry points, one script with subcommands (round 5: the ~30
# one-off tools/gpu_r0*_*.sh, gpu_round.sh, gpu_attr.sh ... scripts of rounds
# 2-5 folded in here; git history keeps the originals the older profiles
# name).  Every GPU step runs under its own timeout and the steps are chained
# so that the first failure ends the call.
#
#   gpurun -- bash tools/gpu.sh tests  <tag> [pytest args...]   GPU tests (default: all of -m gpu)
#   gpurun -- bash tools/gpu.sh round  <tag>                    part A, the NP=2 bench line that reads
#                                                               part A's PMC summary, then part B
#                                                               (round1: without part B)
#   gpurun -- bash tools/gpu.sh parta  <tag>                    tests, smoke, bench lines (Model_1,
#                                                               NP=2, FPSet), NP=2 / FPSet kernel traces
#                                                               + FETCH_SIZE / WRITE_SIZE passes
#   gpurun -- bash tools/gpu.sh partb  <tag>                    NP=3 52-level trace + PMC + bench, the
#                                                               sharded k_claim PMC, the sharded bench
#                                                               line at world 1, per-level costs
#   gpurun -- bash tools/gpu.sh ab-lib <tag> <lib.so>...        same-box NP=2 benches of library builds
#   gpurun -- bash tools/gpu.sh ab-env <tag> "VAR=a" "-" ...    same-box NP=2 benches of env settings
#   gpurun -- bash tools/gpu.sh ab-fpset <tag> "VAR=a" "-" ...  same-box FPSet stress per env setting
#   gpurun -- bash tools/gpu.sh ab-shard <tag> <lib.so>...      warm emulated NP=2 checks (R = 2, 8) per
#                                                               library, then the tlc_order mode's cost
#   gpurun -- bash tools/gpu.sh attr   <tag> [R...]             per-rank, per-level kernel attribution
#                                                               of the emulated sharded NP=2 check
#                                                               (ATTR_ARGS=--first: first-claim mode)
#   gpurun -- bash tools/gpu.sh levels <tag>                    per-level costs (tools/shard_levels.py --np2)
#   gpurun -- bash tools/gpu.sh narrow <tag>                    Model_1 narrow-level phase trace
#                                                               (KC_NARROW_TRACE=1)
#   gpurun -- bash tools/gpu.sh diag   <tag>                    error reports per switch at R = 1, 2, 3
#                                                               (tools/diag_errors.py)
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
# rocprofv3 kernel trace + FETCH_SIZE + WRITE_SIZE passes (separate runs) of
# one command, summarised by tools/pmc_summary.py:  pmc <name> <summary> <cmd...>
pmc() {
  local n=$1 out=$2
  shift 2
  cd /tmp
  step ${n}_trace
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${n}trace -o run -- "$@" > $O/${n}trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/${n}trace.log; return 1; }
  step ${n}_fetch
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${n}fetch -o run -- "$@" > $O/${n}fetch.log 2>&1 || { echo FETCH_FAIL; tail -20 $O/${n}fetch.log; return 1; }
  step ${n}_write
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${n}write -o run -- "$@" > $O/${n}write.log 2>&1 || { echo WRITE_FAIL; tail -20 $O/${n}write.log; return 1; }
  cd $R
  python3 tools/pmc_summary.py --trace $O/${n}trace --fetch $O/${n}fetch --write $O/${n}write $PMC_EXTRA --out $out \
    --command "rocprofv3 -- $(echo "$@" | sed "s#$R/##g")"
}
case "$CMD" in
tests)
  ARGS=${@:-tests -m gpu}
  step tests
  timeout -k 10 1000 python -u -m pytest $ARGS -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo TESTS_FAIL; grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
  ;;
round|round1)
  bash tools/gpu.sh parta $TAG || exit 1
  cp $O/summary.json $R/profiles/${TAG}_np2_rocprof_summary.json
  cp $O/fpset_summary.json $R/profiles/${TAG}_fpset_rocprof_summary.json
  step bench_np2_pmc
  timeout -k 10 600 python -u bench.py > $O/bench_np2_pmc.json 2> $O/bench_np2_pmc.err \
    || { echo BENCH2_FAIL; tail -20 $O/bench_np2_pmc.err; exit 1; }
  cat $O/bench_np2_pmc.json
  [ "$CMD" = round1 ] || bash tools/gpu.sh partb $TAG || exit 1
  ;;
parta)
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
    || { echo GPU_TESTS_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
  step smoke
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
  cat $O/smoke.log
  step bench_model1
  timeout -k 10 300 python -u bench.py --workload model1 --steps 5 --warmup 1 --cpu-seconds 5 > $O/bench_model1.json 2> $O/bench_model1.err \
    || { echo BENCH1_FAIL; tail -20 $O/bench_model1.err; exit 1; }
  cat $O/bench_model1.json
  step bench_np2
  timeout -k 10 600 python -u bench.py > $O/bench_np2.json 2> $O/bench_np2.err || { echo BENCH2_FAIL; tail -20 $O/bench_np2.err; exit 1; }
  cat $O/bench_np2.json
  pmc "" $O/summary.json python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-timing --no-first-claim-line || exit 1
  # FPSet stress (BASELINE config 4): the bench line at 1e10 fps, PMC passes at 2^30
  step bench_fpset
  timeout -k 10 300 python -u bench.py --workload fpset --steps 2 --warmup 1 > $O/bench_fpset.json 2> $O/bench_fpset.err \
    || { echo BENCHF_FAIL; tail -20 $O/bench_fpset.err; exit 1; }
  cat $O/bench_fpset.json
  pmc f $O/fpset_summary.json python3 $R/bench.py --workload fpset --fp-count 1073741824 --steps 1 --warmup 0 || exit 1
  ;;
partb)
  pmc n3 $O/np3_summary.json python3 $R/bench.py --workload np3_52 --steps 1 --warmup 1 --no-cpu-baseline --no-timing \
    --no-first-claim-line || exit 1
  # (the box's copy of profiles/: the bench line below finds this build's PMC)
  cp $O/np3_summary.json $R/profiles/${TAG}_np3_52_rocprof_summary.json
  step bench_np3
  timeout -k 10 400 python -u bench.py --workload np3_52 --steps 3 --warmup 1 --cpu-seconds 10 > $O/bench_np3.json 2> $O/bench_np3.err \
    || { echo NP3_BENCH_FAIL; tail -20 $O/bench_np3.err; exit 1; }
  cat $O/bench_np3.json
  step sharded_pmc
  timeout -k 10 120 python -u tools/sharded_profile.py 8 --out $O/sh_alg.json || { echo ALG_FAIL; exit 1; }
  PMC_EXTRA="--algorithmic $O/sh_alg.json" pmc sh $O/np2_sharded_summary.json python3 $R/tools/sharded_profile.py 8 || exit 1
  cp $O/np2_sharded_summary.json $R/profiles/${TAG}_np2_sharded_rocprof_summary.json
  step bench_sharded
  timeout -k 10 400 python -u bench.py --sharded --steps 3 --warmup 1 --cpu-seconds 10 > $O/bench_np2_sharded_world1.json 2> $O/bench_sharded.err \
    || { echo SHBENCH_FAIL; tail -20 $O/bench_sharded.err; exit 1; }
  cat $O/bench_np2_sharded_world1.json
  bash tools/gpu.sh levels $TAG || exit 1
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
ab-shard)
  LIBS=${@:-tla-kubernetes_amd/kubecheck/lib/libkubecheck.so}
  for rep in 1 2; do
    for L in $LIBS; do
      for RK in 2 8; do
        step "$L R=$RK rep $rep"
        KUBECHECK_LIB=$R/$L timeout -k 10 300 python -u tools/shard_attr.py run $RK --checks 3 >> $O/ab.log 2>&1 \
          || { echo AB_FAIL; tail -20 $O/ab.log; exit 1; }
      done
    done
  done
  for RK in 2 8; do
    step "tlc R=$RK"
    timeout -k 10 300 python -u tools/shard_attr.py run $RK --checks 3 --tlc >> $O/ab.log 2>&1 || { echo TLC_FAIL; tail -20 $O/ab.log; exit 1; }
  done
  grep '^{' $O/ab.log
  ;;
attr)
  # for each R: two checks overlapped (the normal emulation) for wall times,
  # then two with KC_SERIAL=1 under a rocprofv3 kernel + copy trace, and the
  # per-rank / per-kernel / per-level summary of the warm (second) check
  RS=${@:-2 4 8}
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/engine.json 2> $O/engine.err || { echo ENGINE_FAIL; tail -20 $O/engine.err; exit 1; }
  cat $O/engine.json
  for RK in $RS; do
    step "R=$RK"
    timeout -k 10 300 python -u tools/shard_attr.py run $RK --checks 3 $ATTR_ARGS > $O/wall_R$RK.log 2>&1 || { echo WALL_FAIL; tail -20 $O/wall_R$RK.log; exit 1; }
    cat $O/wall_R$RK.log
    cd /tmp
    KC_SERIAL=1 timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace_R$RK -o run -- python3 $R/tools/shard_attr.py run $RK --checks 2 $ATTR_ARGS > $O/serial_R$RK.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/serial_R$RK.log; exit 1; }
    cd $R
    grep '^{' $O/serial_R$RK.log
    python3 tools/shard_attr.py summarize $O/trace_R$RK $RK --out $O/attr_R$RK.json > /dev/null || exit 1
    python3 -c "import json;d=json.load(open('$O/attr_R$RK.json'));print({k:d[k] for k in ('span_ms','sum_over_ranks_ms','max_rank_ms','unattributed_ms')});[print('  %-44s %9.3f %9.3f %6d'%(n,v['sum'],v['max_rank'],v['calls'])) for n,v in list(d['per_kernel_ms'].items())[:22]]"
    rm -rf $O/trace_R$RK
  done
  ;;
levels)
  step levels
  timeout -k 10 400 python -u tools/shard_levels.py --np2 > $O/shard_levels.log 2>&1 \
    || { echo LEVELS_FAIL; tail -30 $O/shard_levels.log; exit 1; }
  grep '^{' $O/shard_levels.log
  ;;
narrow)
  step narrow_trace
  KC_NARROW_TRACE=1 timeout -k 10 200 python -u -c "
import sys, time; sys.path.insert(0, 'tla-kubernetes_amd')
import torch
from kubecheck import ModelChecker, ModelConfig
mc = ModelChecker(ModelConfig())
for k in range(3):
    t = time.perf_counter(); r = mc.run(); print('check', k, round((time.perf_counter() - t) * 1e3, 3), 'ms', r.distinct, r.depth, flush=True)
" > $O/ntrace.log 2>&1 || { echo NTRACE_FAIL; tail -20 $O/ntrace.log; exit 1; }
  tail -2 $O/ntrace.log
  ;;
diag)
  step diag
  timeout -k 10 300 python -u tools/diag_errors.py 1 2 3 > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag.log; exit 1; }
  grep '^{' $O/diag.log
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
  sed -n 1,30p tools/gpu.sh
  exit 2
  ;;
esac
step done
