# Shard-path iteration: sharded parity tests (emulated ranks, RCCL world 1),
# the gloo-free native sharded NP=2 bench at world 1 and with RCCL forced at
# world 1, and the engine bench beside it.   gpurun -- bash tools/gpu_shard_iter.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for round in 1 2; do
  timeout -k 10 300 python -u bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline > $O/sh_$round.json 2> $O/sh_$round.err || { echo SH_FAIL; tail -20 $O/sh_$round.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sh_$round.json')); print('sharded world1', d['ms_per_step'])"
  KC_RCCL_FORCE=1 timeout -k 10 300 python -u bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline > $O/shf_$round.json 2> $O/shf_$round.err || { echo SHF_FAIL; tail -20 $O/shf_$round.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/shf_$round.json')); print('sharded world1 RCCL forced', d['ms_per_step'])"
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/en_$round.json 2> $O/en_$round.err || { echo EN_FAIL; tail -20 $O/en_$round.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/en_$round.json')); print('engine', d['ms_per_step'])"
done
