# Where k_claim's waves spend their cycles (one NP=2 bench check): one PMC
# pass of 8 SQ counters (wave cycles, waiting on anything / on instruction
# issue, active instruction cycles by unit), summed over k_claim launches.
#   gpurun -- bash tools/gpu_r04_stall.sh <tag>
set -o pipefail
TAG=${1:-r04s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CU_CYCLES"
timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-timing > $O/p1.log 2>&1 || { echo PMC_FAIL; tail -5 $O/p1.log; exit 1; }
cd $R
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(O + "/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = "k_claim" if "k_claim<" in n else ("k_settle_rec" if "k_settle_rec" in n else None)
        if k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    wc = v["SQ_WAVE_CYCLES"]
    print(k, {c: f"{x:.4g}" for c, x in sorted(v.items())})
    print("  per wave-cycle:", {c: round(x / wc, 3) for c, x in sorted(v.items()) if c != "SQ_WAVE_CYCLES"})
PY
