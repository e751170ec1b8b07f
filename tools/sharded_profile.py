"""One sharded NP=2 check with R ranks emulated on one GPU (LocalComm; the
N-GPU protocol's kernels, k_claim<..., SH=true> among them), for rocprofv3
kernel-trace / PMC passes; prints the algorithmic bytes of k_claim over all
ranks and launches (kubecheck.distributed.claim_alg_bytes: the engine's model
of SURVEY §8(d) — parents x S, generated successors x 64, the deferred
rebuild — plus the staged records), which tools/pmc_summary.py's output is
divided by to get the PMC/algorithmic ratio that bench.py applies to the
N-GPU line's k_claim.  The claims are first-claim (the sharded bench's
default) unless --deterministic.

  python tools/sharded_profile.py [R] [--deterministic] [--out file.json]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))
import torch  # noqa: E402,F401

from kubecheck import ModelConfig, Spec  # noqa: E402
from kubecheck.distributed import NativeShardedChecker, claim_alg_bytes  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 8
first = "--deterministic" not in sys.argv
cfg = ModelConfig(np=2, keep_trace=False, timing=2, first_claim=first)
mc = NativeShardedChecker(cfg, emulate=R)
try:
    r = mc.run()
    ms, launches, parents = mc.claim_times()
    sh = [mc.shard_result(i) for i in range(R)]
    gen = sum(x["generated"] for x in sh)
    dfr = sum(x["deferred"] for x in sh)
    records = mc.records_sent
    rb = mc.record_bytes
finally:
    mc.close()
S = 8 * Spec(cfg).state_words
alg = claim_alg_bytes(parents, gen, dfr, records, S, rb)
out = {"ranks": R, "claims": "first" if first else "deterministic", "claim_mode": r.get("claim_mode"),
       "distinct": r["distinct"], "k_claim_launches": launches, "k_claim_ms": round(ms, 3),
       "parents": parents, "generated": gen, "deferred": dfr, "records": records, "record_bytes": rb,
       "algorithmic_bytes": alg, "stream_read_bytes": parents * S,
       "algorithmic_bytes_per_launch": alg / max(launches, 1),
       "stream_read_bytes_per_launch": parents * S / max(launches, 1)}
print(json.dumps(out), flush=True)
if "--out" in sys.argv:
    json.dump(out, open(sys.argv[sys.argv.index("--out") + 1], "w"), indent=1)
