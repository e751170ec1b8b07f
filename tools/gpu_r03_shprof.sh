# PMC profile of the sharded k_claim (8 emulated ranks, NP=2): kernel trace +
# FETCH_SIZE + WRITE_SIZE passes, summarised with the run's algorithmic bytes.
#   gpurun -- bash tools/gpu_r03_shprof.sh <tag>
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/sharded_profile.py 8 --out $O/sh_alg.json || { echo ALG_FAIL; exit 1; }
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shtrace -o run -- python3 $R/tools/sharded_profile.py 8 > $O/shtrace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/shtrace.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/shfetch -o run -- python3 $R/tools/sharded_profile.py 8 > $O/shfetch.log 2>&1 || { echo FETCH_FAIL; tail -20 $O/shfetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/shwrite -o run -- python3 $R/tools/sharded_profile.py 8 > $O/shwrite.log 2>&1 || { echo WRITE_FAIL; tail -20 $O/shwrite.log; exit 1; }
cd $R
python3 tools/pmc_summary.py --trace $O/shtrace --fetch $O/shfetch --write $O/shwrite --algorithmic $O/sh_alg.json --out $O/np2_sharded_summary.json --command "rocprofv3 -- python3 tools/sharded_profile.py 8 (NP=2, 8 ranks emulated on one GPU)"
echo "== done $(date +%T)"
