# The NP=3 52-level golden (tests/golden/np3_52levels.json) on a GPU box's
# host: the oracle's multi-threaded BFS with 128-bit keys (two independent
# 64-bit hashes of the packed canonical words, one 16-B compare-exchange per
# probe), 16 threads, a 2^32-slot (64 GiB) set; ~120 GB of host RAM.
# Its first 40 levels equal the sequential oracle's tests/golden/np3_40levels.json.
#   bash tools/np3_golden.sh <out.json>
set -o pipefail
OUT=${1:-gpurun_out/np3_52levels.json}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
timeout -k 10 1000 $R/oracle/build/kubeapi_oracle -np 3 -maxlevels 52 -threads 16 -fp128 -fpsetlog2 32 > $OUT.tmp || exit 1
python3 - "$OUT.tmp" "$OUT" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
d["generator"] = ("tools/np3_golden.sh: oracle/build/kubeapi_oracle -np 3 -maxlevels 52 -threads 16 -fp128 "
                  "-fpsetlog2 32 (oracle/kubeapi_oracle.c ko_bench_parallel, 128-bit keys)")
json.dump(d, open(sys.argv[2], "w"), indent=1)
PY
rm -f $OUT.tmp
