set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload model1 --steps 5 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_model1.json 2> gpurun_out/bench_model1.err || { echo FAIL1; tail -20 gpurun_out/bench_model1.err; exit 1; }
cat gpurun_out/bench_model1.json
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_np2.json 2> gpurun_out/bench_np2.err || { echo FAIL2; tail -20 gpurun_out/bench_np2.err; exit 1; }
cat gpurun_out/bench_np2.json
