# Same-box A/B of the FPSet stress (BASELINE config 4): speculative first
# CAS (default) vs load-first (KC_FPSET_SPEC=0), 50% and 75% load; then the
# FPSet parity tests.   gpurun -- bash tools/gpu_ab_fpset.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fpset.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for round in 1 2; do
  for v in 1 0; do
    KC_FPSET_SPEC=$v timeout -k 10 300 python -u bench.py --workload fpset --steps 1 --warmup 1 > $O/f_${v}_$round.json 2> $O/f_${v}_$round.err || { echo BENCH_FAIL; tail -20 $O/f_${v}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/f_${v}_$round.json')); c=d['config']; print('spec=$v', $round, round(c['inserts_per_s']/1e9,2), round(c['lookups_per_s']/1e9,2), d['ms_per_step'])"
  done
done
KC_FPSET_SPEC=1 timeout -k 10 300 python -u bench.py --workload fpset --steps 1 --warmup 1 --fp-load 0.75 > $O/f75.json 2> $O/f75.err || { echo BENCH_FAIL; tail -20 $O/f75.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/f75.json')); c=d['config']; print('spec 75%', round(c['inserts_per_s']/1e9,2), round(c['lookups_per_s']/1e9,2))"
