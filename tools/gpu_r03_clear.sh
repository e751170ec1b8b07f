# ClaimSet per-run clear: hipMemsetAsync vs the k_claimset_clear kernel at
# several grid sizes; kernel durations from a trace, then a same-box bench A/B.
set -o pipefail
TAG=${1:-r03ap}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing"
for m in memset kernel:1024 kernel:2048 kernel:4096 kernel:8192; do
  n=$(echo $m | tr ':' '_')
  KC_CS_CLEAR=$m timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o run -- python3 $B > $O/$n.log 2>&1 || { echo TRACE_FAIL $m; tail -20 $O/$n.log; exit 1; }
  python3 - $O/$n $m <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in csv.DictReader(open(f))
     if ("fillBuffer" in r["Kernel_Name"] or "k_claimset_clear" in r["Kernel_Name"])]
big = [x for x in d if x > 5]
print(sys.argv[2], "64 GiB clears (ms):", [round(x, 2) for x in big])
PY
done
cd $R
bash tools/gpu_r03_env_ab.sh $TAG KC_CS_CLEAR=memset -
