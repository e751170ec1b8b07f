# VALU lane utilisation of the k_claim ablation variants (KC_ABLATE=1, ABL 0..5):
# which SQ counters this rocprofv3 offers, then one PMC pass over them,
# summed per kernel template (ABL 0..3).
set -o pipefail
TAG=${1:-r04v}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || { echo LIST_FAIL; tail -5 $O/avail.txt; exit 1; }
want="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
have=""
for c in $want; do grep -q "\b$c\b" $O/avail.txt && have="$have $c"; done
echo "counters:$have"
KC_ABLATE=1 timeout -s KILL 300 rocprofv3 --pmc $have --output-format csv -d $O/p1 -o run -- python3 $R/tools/exp_run.py --np 2 --runs 1 > $O/p1.log 2>&1 || { echo PMC_FAIL; tail -5 $O/p1.log; exit 1; }
cd $R
python3 - "$O" <<'PY'
import csv, glob, sys, re, collections
O = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(O + "/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "k_claim" not in n and "k_emit" not in n:
            continue
        m = re.search(r"k_claim<kc::Model<[^>]*>, (\d)", n)
        k = ("k_claim ABL" + m.group(1)) if m else re.sub(r"\(.*$", "", n)[:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    lanes = v.get("SQ_THREAD_CYCLES_VALU", 0) / max(v.get("SQ_INSTS_VALU", 1), 1)
    print(k, f"lanes/VALU {lanes:.1f}", {c: f"{x:.5g}" for c, x in sorted(v.items())})
PY
