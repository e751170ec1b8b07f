# PMC passes over one tools/exp_run.py run (one counter group per rocprofv3 run)
set -o pipefail
TAG=${1:-p}
shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
n=0
for grp in "$@"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$n -o run -- python3 $R/tools/exp_run.py --runs 1 > $O/p$n.log 2>&1 || { echo PMC_FAIL $grp; tail -5 $O/p$n.log; exit 1; }
done
cd $R
python3 - "$O" <<'PY'
import csv, glob, sys, re, collections
O = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"<.*", "", re.sub(r"\(.*$", "", r["Kernel_Name"])).replace("void ", "").split("::")[-1]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k in ("k_claim", "k_settle_rec", "k_emit"):
    if k in agg:
        print(k, {c: f"{v:.4g}" for c, v in sorted(agg[k].items())})
PY
