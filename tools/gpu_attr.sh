# Attribution of the emulated sharded NP=2 check (tools/shard_attr.py): for
# each R, two checks overlapped (the normal emulation) for wall times, then
# two checks with KC_SERIAL=1 under a rocprofv3 kernel + copy trace, and the
# per-rank / per-kernel summary of the warm (second) check.
#   gpurun -- bash tools/gpu_attr.sh <tag> [R ...]
set -o pipefail
TAG=${1:-attr}
shift
RS=${@:-2 4 8}
R0=$GRAFT_REPO_ROOT
O=$R0/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R0
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/engine.json 2> $O/engine.err || { echo ENGINE_FAIL; tail -20 $O/engine.err; exit 1; }
cat $O/engine.json
for R in $RS; do
  echo "== R=$R $(date +%T)"
  timeout -k 10 300 python -u tools/shard_attr.py run $R --checks 3 > $O/wall_R$R.log 2>&1 || { echo WALL_FAIL; tail -20 $O/wall_R$R.log; exit 1; }
  cat $O/wall_R$R.log
  cd /tmp
  KC_SERIAL=1 timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace_R$R -o run -- python3 $R0/tools/shard_attr.py run $R --checks 2 > $O/serial_R$R.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/serial_R$R.log; exit 1; }
  cd $R0
  grep '^{' $O/serial_R$R.log
  python3 tools/shard_attr.py summarize $O/trace_R$R $R --out $O/attr_R$R.json > /dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/attr_R$R.json'));print({k:d[k] for k in ('span_ms','sum_over_ranks_ms','max_rank_ms','unattributed_ms')});[print('  %-44s %9.3f %9.3f %6d'%(n,v['sum'],v['max_rank'],v['calls'])) for n,v in list(d['per_kernel_ms'].items())[:22]]"
  rm -rf $O/trace_R$R
done
echo "== done $(date +%T)"
