# rocprofv3 kernel trace of tools/exp_sharded.py (sharded NP=2 at world 1)
set -o pipefail
TAG=${1:-ts}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/exp_sharded.py --runs 2 > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.log; exit 1; }
grep distinct $O/trace.log
cd $R
python3 tools/pmc_summary.py --trace $O/trace --out $O/summary.json
