# Same-box A/B of library builds (KUBECHECK_LIB): NP=2 bench, interleaved.
#   gpurun -- bash tools/gpu_r03_ab_lib.sh <tag> <lib1> <lib2> ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
B="python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
for rep in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    echo "== $n $rep $(date +%T)"
    KUBECHECK_LIB=$R/$L timeout -k 10 300 $B > $O/${n}_$rep.json 2> $O/${n}_$rep.err || { echo "B_FAIL"; tail -20 $O/${n}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${n}_$rep.json'));print(d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'])"
  done
done
echo "== done $(date +%T)"
