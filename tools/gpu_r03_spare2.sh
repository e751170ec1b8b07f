# Spare ClaimSet, clear kicked at the first wide chunk: trace (when the clear
# runs) and same-box bench A/B over the clear's workgroup count and in-place.
set -o pipefail
TAG=${1:-r03am}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing"
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/spare -o run -- python3 $B > $O/spare.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/spare.log; exit 1; }
cd $R
python3 - $O/spare <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50]) for r in csv.DictReader(open(f)))
t0 = ks[0][0]
starts = [k[0] for k in ks if "insert_list" in k[2]]
print("run lengths ms", [round((b - a) / 1e6, 1) for a, b in zip(starts, starts[1:])])
for s, e, n in ks:
    if "k_claimset_clear" in n:
        ov = sum(max(0, min(e, e2) - max(s, s2)) for s2, e2, n2 in ks if "k_claim<" in n2) / 1e6
        print("clear at %.1f ms, %.2f ms long, overlaps k_claim %.2f ms" % ((s - t0) / 1e6, (e - s) / 1e6, ov))
PY
bash tools/gpu_r03_env_ab.sh $TAG - KC_CS_SPARE=0 KC_CS_CLEAR_WG=16 KC_CS_CLEAR_WG=256
