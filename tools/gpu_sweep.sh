set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for ch in 0 2097152 524288 262144; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --chunk $ch > gpurun_out/sweep_$ch.json 2> gpurun_out/sweep_$ch.err || { echo FAIL $ch; tail -5 gpurun_out/sweep_$ch.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep_$ch.json')); print($ch, d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['config']['chunks'])"
done
