set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for ch in 2097152 262144 65536; do
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --chunk $ch > gpurun_out/sweep_$ch.json 2> gpurun_out/sweep_$ch.err || { echo FAIL $ch; tail -5 gpurun_out/sweep_$ch.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep_$ch.json')); print($ch, d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['config']['fpset_probes'], d['config']['chunks'])"
done
