"""One sharded NP=2 check with R ranks emulated on one GPU (LocalComm; the
N-GPU protocol's kernels, k_claim<..., SH=true> among them), for rocprofv3
kernel-trace / PMC passes; prints the algorithmic bytes of k_claim (parents
x S + generated successors x 64) over all ranks and launches,
which tools/pmc_summary.py's output is divided by to get the PMC/algorithmic
ratio that bench.py applies to the N-GPU line's k_claim.

  python tools/sharded_profile.py [R] [--out file.json]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))
import torch  # noqa: E402,F401

from kubecheck import ModelConfig, Spec  # noqa: E402
from kubecheck.distributed import NativeShardedChecker  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 8
cfg = ModelConfig(np=2, keep_trace=False, timing=2)
mc = NativeShardedChecker(cfg, emulate=R)
try:
    r = mc.run()
    ms, launches, parents = mc.claim_times()
    gen = sum(mc.shard_result(i)["generated"] for i in range(R))
finally:
    mc.close()
S = 8 * Spec(cfg).state_words
out = {"ranks": R, "distinct": r["distinct"], "k_claim_launches": launches, "k_claim_ms": round(ms, 3),
       "algorithmic_bytes": parents * S + gen * 64, "stream_read_bytes": parents * S,
       "algorithmic_bytes_per_launch": (parents * S + gen * 64) / max(launches, 1),
       "stream_read_bytes_per_launch": parents * S / max(launches, 1)}
print(json.dumps(out), flush=True)
if "--out" in sys.argv:
    json.dump(out, open(sys.argv[sys.argv.index("--out") + 1], "w"), indent=1)
