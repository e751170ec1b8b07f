set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_np2.json 2> gpurun_out/bench_np2.err || { echo FAIL2; tail -20 gpurun_out/bench_np2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_np2.json')); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['roofline'])"
