"""A/B for VERDICT r2 item 6 (locality of k_claim's random probes): the SAME
work with the ClaimSet at different sizes.  A table that fits the MALL
(Infinity Cache, 256 MB) or a few GB shows what address locality could buy
k_claim at best: region-partitioning the probes can at most shrink the
window they hit to such a size, and it costs an extra pass over every tile
representative.  Prints one JSON line per (workload, table size): k_claim
ms (HIP events), probes and ns per probe.

  python tools/locality_ab.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import torch  # noqa: E402,F401

from kubecheck import ModelChecker, ModelConfig  # noqa: E402


def measure(kw, slots, reps=3):
    mc = ModelChecker(ModelConfig(**kw, fpset_slots=slots, timing=2, keep_trace=False))
    try:
        mc.run()
        best = None
        for _ in range(reps):
            r = mc.run()
            kt = mc.kernel_times()
            cur = (kt["expand"][0], r)
            best = cur if best is None or cur[0] < best[0] else best
        ms, r = best
        return {"slots": slots, "table_MiB": slots * 16 >> 20, "fpset_slots_final": r.fpset_slots,
                "claim_ms": round(ms, 3), "probes": r.fpset_probes, "distinct": r.distinct,
                "ns_per_probe": round(ms * 1e6 / max(r.fpset_probes, 1), 4), "check_ms": round(r.seconds * 1e3, 2)}
    finally:
        mc.close()


def main():
    if "--full-only" in sys.argv:
        for s in (1 << 31, 1 << 32, 1 << 31, 1 << 32):
            out = measure(dict(np=2), s, reps=2)
            out["workload"] = "np2 full"
            print(json.dumps(out), flush=True)
        return
    # the NP=2 model's first 60 levels (~1.2e8 states): tables of 4 GiB .. 64 GiB
    for L, sizes in ((60, (1 << 28, 1 << 29, 1 << 31, 1 << 32)),):
        for s in sizes:
            out = measure(dict(np=2, max_levels=L), s)
            out["workload"] = f"np2 first {L} levels"
            print(json.dumps(out), flush=True)
    # the whole NP=2 model: the natural 32 GiB table against 64 GiB
    for s in (1 << 31, 1 << 32):
        out = measure(dict(np=2), s, reps=2)
        out["workload"] = "np2 full"
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
