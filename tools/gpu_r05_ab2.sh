# Round 5: warm emulated NP=2 checks per library build and mode (same box):
# R = 2 / 8 with the default library and the 5-waves-per-EU sharded k_claim
# variant, then the TLC-ordered mode's cost at R = 2 / 8.
#   gpurun -- bash tools/gpu_r05_ab2.sh <tag> [lib ...]
set -o pipefail
TAG=${1:-r05n}
shift
R0=$GRAFT_REPO_ROOT
cd $R0
O=$R0/gpurun_out/$TAG
mkdir -p $O
LIBS=${@:-tla-kubernetes_amd/kubecheck/lib/libkubecheck.so}
for rep in 1 2; do
  for L in $LIBS; do
    for R in 2 8; do
      echo "== $L R=$R rep $rep $(date +%T)"
      KUBECHECK_LIB=$R0/$L timeout -k 10 300 python -u tools/shard_attr.py run $R --checks 3 >> $O/ab.log 2>&1 \
        || { echo AB_FAIL; tail -20 $O/ab.log; exit 1; }
    done
  done
done
for R in 2 8; do
  echo "== tlc R=$R $(date +%T)"
  timeout -k 10 300 python -u tools/shard_attr.py run $R --checks 3 --tlc >> $O/ab.log 2>&1 || { echo TLC_FAIL; tail -20 $O/ab.log; exit 1; }
done
grep '^{' $O/ab.log
