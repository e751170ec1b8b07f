# Kernel trace of the NP=2 bench with the spare ClaimSet (side-stream clear)
# and without (KC_CS_SPARE=0): when the 64 GiB clear runs against k_claim.
set -o pipefail
TAG=${1:-r03ak}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing"
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/spare -o run -- python3 $B > $O/spare.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/spare.log; exit 1; }
KC_CS_SPARE=0 timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/inplace -o run -- python3 $B > $O/inplace.log 2>&1 || { echo TRACE2_FAIL; tail -20 $O/inplace.log; exit 1; }
cd $R
for m in spare inplace; do
python3 - $O/$m <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40], r.get("Queue_Id", "")) for r in rows))
t0 = ks[0][0]
fills = [k for k in ks if "fillBuffer" in k[2] and k[1] - k[0] > 2e6]
print(sys.argv[1].split("/")[-1], "kernels", len(ks), "span ms %.1f" % ((ks[-1][1] - t0) / 1e6))
for s, e, n, q in fills:
    ov = sum(max(0, min(e, e2) - max(s, s2)) for s2, e2, n2, q2 in ks if "k_claim" in n2) / 1e6
    print("  fill q%s at %.1f ms, %.2f ms long, overlaps k_claim %.2f ms" % (q, (s - t0) / 1e6, (e - s) / 1e6, ov))
PY
done
