# Round-4 host probe: is there a JVM / tla2tools.jar
# on the GPU box, and the CPU comparator over the whole NP=2 model at the
# box's full affinity count, 128, 64 and 16 threads.  Then the GPU tests.
#   gpurun -- bash tools/gpu_r04_probe.sh <tag>
set -o pipefail
TAG=${1:-r04a}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step jvm
{
  echo "command -v java:"; command -v java || echo "  (none)"
  echo "java -version:"; java -version 2>&1 || echo "  (no java)"
  echo "JAVA_HOME=${JAVA_HOME:-unset}"
  echo "ls /usr/lib/jvm:"; ls /usr/lib/jvm 2>&1 || true
  echo "find / -xdev -name 'tla2tools*.jar' (timeout 120 s):"
  timeout 120 find / -xdev -name 'tla2tools*.jar' 2>/dev/null || true
  echo "find / -xdev -name 'java' -type f (timeout 120 s):"
  timeout 120 find / -xdev -name 'java' -type f 2>/dev/null || true
  echo "end of probe"
} > $O/jvm_probe.log 2>&1
cat $O/jvm_probe.log
step cpus
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; grep -m1 "model name" /proc/cpuinfo; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; free -g; } > $O/cpus.log 2>&1
cat $O/cpus.log
AFF=$(python3 -c "import os; print(len(os.sched_getaffinity(0)))")
for T in $AFF 128 64 16; do
  step "cpu comparator, whole NP=2, $T threads"
  timeout -k 10 400 $R/oracle/build/kubeapi_oracle -np 2 -threads $T -fpsetlog2 31 > $O/cpu_np2_full_t$T.json 2> $O/cpu_np2_full_t$T.err || { echo CPU_FAIL; tail $O/cpu_np2_full_t$T.err; exit 1; }
  cat $O/cpu_np2_full_t$T.json
done
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
step bench
timeout -k 10 300 python -u bench.py --steps 5 --cpu-seconds 5 > $O/bench_np2.json 2> $O/bench_np2.err || { echo BENCH_FAIL; tail -20 $O/bench_np2.err; exit 1; }
cat $O/bench_np2.json
step done
