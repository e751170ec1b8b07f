# Same-box A/B of environment settings on the NP=2 bench (interleaved twice).
#   gpurun -- bash tools/gpu_r03_env_ab.sh <tag> "VAR=a" "VAR=b" ...   ("-" = no setting)
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
B="python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
i=0
for rep in 1 2; do
  for v in "$@"; do
    i=$((i+1))
    echo "== [$v] $rep $(date +%T)"
    if [ "$v" = "-" ]; then E=""; else E="$v"; fi
    env $E timeout -k 10 300 $B > $O/run_$i.json 2> $O/run_$i.err || { echo "B_FAIL"; tail -20 $O/run_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/run_$i.json'));c=d['config'];print(d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'], 'settle_reads', c['settle_reads'])"
  done
done
echo "== done $(date +%T)"
