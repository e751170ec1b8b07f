set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke1.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke1.log; exit 1; }
cat gpurun_out/smoke1.log
