# PMC calibration (tools/microbench/pmc_calib.hip): per-shape FETCH_SIZE /
# WRITE_SIZE per access.  gpurun -- bash tools/gpu_pmc_calib.sh <tag> [counters...]
set -o pipefail
TAG=${1:-r02b}
shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
B=$R/tools/microbench/pmc_calib
cd /tmp
if [ $# -eq 0 ]; then
  echo "== avail $(date +%T)"
  timeout -s KILL 120 rocprofv3 -L > $O/avail.txt 2>&1 || echo "list-avail rc=$?"
  echo "== plain $(date +%T)"
  timeout -k 10 120 $B > $O/plain.log 2>&1 || { echo PLAIN_FAIL; cat $O/plain.log; exit 1; }
  cat $O/plain.log
  set -- FETCH_SIZE WRITE_SIZE
fi
for C in "$@"; do
  echo "== pmc $C $(date +%T)"
  timeout -s KILL 120 rocprofv3 --pmc ${C//,/ } --output-format csv -d $O/pmc_${C//,/_} -o run -- $B > $O/pmc_${C//,/_}.log 2>&1 || { echo "PMC_FAIL $C"; tail -20 $O/pmc_${C//,/_}.log; exit 1; }
done
echo "== done $(date +%T)"
