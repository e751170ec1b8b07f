# Round 5: the sharded GPU tests, the error-report diagnostic per switch and
# the R = 8 attribution, in one call.
#   gpurun -- bash tools/gpu_r05_tests.sh <tag>
set -o pipefail
TAG=${1:-r05f}
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/diag_errors.py 1 2 3 > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag.log; exit 1; }
grep '^{' $O/diag.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['R'], ','.join(k+'='+v for k,v in d['env'].items()), d['case'], d['error'], d['level'], d['want_level'], d['widths_ok'])"
KC_TESTS="tests/test_gpu_shard.py tests/test_gpu_hostcomm.py tests/test_gpu_shard_seenspill.py" bash tools/gpu_shard_tests.sh $TAG 8 || exit 1
