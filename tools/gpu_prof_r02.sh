# Round-2 profiles: for each bench workload a rocprofv3 kernel trace + stats
# pass, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (one counter
# group per run, MI355X_MICROARCH.md §HBM), summarised by tools/pmc_summary.py
# into gpurun_out/<tag>/<workload>_rocprof_summary.json.  Then (optionally)
# the multi-core CPU comparator over the WHOLE NP=2 model.
#   gpurun -- bash tools/gpu_prof_r02.sh <tag> "np2 fpset model1" [cpu]
set -o pipefail
TAG=${1:-r02p}
WL=${2:-"np2 fpset model1"}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
for w in $WL; do
  case $w in
    np2) B="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline"; PMC=1;;
    fpset) B="$R/bench.py --workload fpset --steps 1 --warmup 0"; PMC=1;;
    model1) B="$R/bench.py --workload model1 --steps 3 --warmup 1 --no-cpu-baseline"; PMC=0;;
    *) echo "unknown workload $w"; exit 1;;
  esac
  step "$w trace"
  (cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$w/trace -o run -- python3 $B > $O/$w.trace.log 2>&1) || { echo TRACE_FAIL $w; tail -20 $O/$w.trace.log; exit 1; }
  ARGS="--trace $O/$w/trace"
  if [ $PMC = 1 ]; then
    step "$w fetch"
    (cd /tmp && timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$w/fetch -o run -- python3 $B > $O/$w.fetch.log 2>&1) || { echo FETCH_FAIL $w; tail -20 $O/$w.fetch.log; exit 1; }
    step "$w write"
    (cd /tmp && timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$w/write -o run -- python3 $B > $O/$w.write.log 2>&1) || { echo WRITE_FAIL $w; tail -20 $O/$w.write.log; exit 1; }
    ARGS="$ARGS --fetch $O/$w/fetch --write $O/$w/write"
  fi
  python3 $R/tools/pmc_summary.py $ARGS --out $O/${w}_rocprof_summary.json --command "rocprofv3 ... -- python3 bench.py ${B#$R/bench.py }" || exit 1
  # keep the stats CSV, drop the bulky per-dispatch traces
  find $O/$w -name "*kernel_stats.csv" -exec cp {} $O/${w}_kernel_stats.csv \; || true
  rm -rf $O/$w
done
if [ "$3" = cpu ]; then
  step "cpu comparator (whole NP=2 model, 16 threads)"
  timeout -k 10 900 $R/oracle/build/kubeapi_oracle -np 2 -threads 16 -budget 800 -fpsetlog2 31 > $O/cpu_np2_full.json 2> $O/cpu_np2_full.err || { echo CPU_FAIL; tail $O/cpu_np2_full.err; exit 1; }
  grep -m1 "model name" /proc/cpuinfo >> $O/cpu_np2_full.err
  cat $O/cpu_np2_full.json
fi
step done
