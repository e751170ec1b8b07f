"""Per-level fixed cost of the native sharded loop (kc_group_*), for DESIGN §6:
seconds per check and microseconds per BFS level, with R ranks emulated on
one GPU (LocalComm) and with RCCL at world 1 (KC_RCCL_FORCE=1 keeps the
world-1 collectives on RCCL), next to the single-GPU engine.

  python tools/shard_levels.py [--np2] [--ab]

--ab adds the same runs with KC_SNARROW=0 (no device-driven narrow levels:
every level on the counted path).  Every run also reports RCCL world 1 with
its identity collectives (the solo levels: one host sync per level) and the
one-rank emulation with KC_SOLO=0 (the gather path at world 1)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import torch  # noqa: E402,F401  (owns the HIP runtime first)

from kubecheck import ModelChecker, ModelConfig  # noqa: E402
from kubecheck.distributed import NativeShardedChecker  # noqa: E402


def timed(make, reps):
    mc = make()
    try:
        mc.run()                                  # warm (allocations, table growth)
        t0 = time.perf_counter()
        for _ in range(reps):
            r = mc.run()
        dt = (time.perf_counter() - t0) / reps
    finally:
        mc.close()
    depth = r["depth"] if isinstance(r, dict) else r.depth
    distinct = r["distinct"] if isinstance(r, dict) else r.distinct
    return {"ms": round(dt * 1e3, 3), "levels": depth, "us_per_level": round(dt * 1e6 / depth, 1),
            "distinct": distinct}


def main():
    out = {}
    models = [("model1", {}, 5)]
    if "--np2" in sys.argv:
        models.append(("np2", dict(np=2, keep_trace=False), 2))
    modes = [("", None)] + ([("_counted", "0")] if "--ab" in sys.argv else [])
    for name, kw, reps in models:
        out[f"{name}_engine"] = timed(lambda: ModelChecker(ModelConfig(**kw)), reps)
        for tag, sn in modes:
            if sn is not None:
                os.environ["KC_SNARROW"] = sn
            for R in (1, 2, 8):
                out[f"{name}_emulated_R{R}{tag}"] = timed(
                    lambda: NativeShardedChecker(ModelConfig(**kw), emulate=R), reps)
            os.environ["KC_RCCL_FORCE"] = "1"
            out[f"{name}_rccl_world1{tag}"] = timed(lambda: NativeShardedChecker(ModelConfig(**kw), 0, 1), reps)
            del os.environ["KC_RCCL_FORCE"]
            out[f"{name}_world1_solo{tag}"] = timed(lambda: NativeShardedChecker(ModelConfig(**kw), 0, 1), reps)
            os.environ["KC_SOLO"] = "0"
            out[f"{name}_emulated_R1_nosolo{tag}"] = timed(
                lambda: NativeShardedChecker(ModelConfig(**kw), emulate=1), reps)
            del os.environ["KC_SOLO"]
            os.environ.pop("KC_SNARROW", None)
            print(json.dumps({k: v for k, v in out.items() if k.startswith(name)}), flush=True)


if __name__ == "__main__":
    main()
