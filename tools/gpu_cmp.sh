set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/cmpb; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for B in 2 1 4; do
  if [ $B = 2 ]; then L=""; else L=$R/tla-kubernetes_amd/kubecheck/lib/exp/libkc_b$B.so; fi
  KUBECHECK_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b$B.json 2> $O/b$B.err || { echo BENCH_FAIL; tail -20 $O/b$B.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$B.json'));print('B=$B',d['ms_per_step'],d['kernel_ms_per_step'])"
done
