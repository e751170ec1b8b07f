"""How many different action bodies a k_claim wave runs per successor trip
(DESIGN §7.3): on levels of the NP=2 model captured by the GPU engine, in
the frontier's own order, sampled tiles of 256 parents are dealt to four
64-lane waves three ways — lane = parent (round 2), by successor count (the
round-3 deal), by successor count then action sequence — and for each wave
and trip t the distinct actions of the lanes' t-th successors are counted.
A wave runs one action body per distinct action (divergence), so the sum is
the serialised body count; lane trips / (64 x wave trips) is the busy share.

  python tools/divergence_study.py [levels...]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import torch  # noqa: E402,F401

import kubecheck  # noqa: E402
from kubecheck import ModelChecker, ModelConfig  # noqa: E402


def wave_cost(seqs):
    """seqs: 64 action sequences (one lane each) -> (wave trips, bodies, lane trips)"""
    trips = max((len(s) for s in seqs), default=0)
    bodies = 0
    for t in range(trips):
        bodies += len({s[t] for s in seqs if len(s) > t})
    return trips, bodies, sum(len(s) for s in seqs)


def main():
    levels = [int(x) for x in sys.argv[1:]] or [50, 86, 120]
    lib = kubecheck.load()
    cfg = ModelConfig(np=2)
    c = cfg.to_c()
    acts = (C.c_int * 64)()
    fa = C.c_int()
    rng = np.random.RandomState(11)
    for L in levels:
        with ModelChecker(ModelConfig(np=2, max_levels=L + 1, keep_trace=False)) as mc:
            mc.capture_level(L)
            mc.run()
            tups = mc.level_tuples(L)
        tw = tups.shape[1]
        out = (C.c_uint64 * (64 * tw))()
        ntiles = len(tups) // 256
        pick = rng.choice(ntiles, min(ntiles, 300), replace=False)
        tot = {"lane=parent": [0, 0, 0], "by count": [0, 0, 0], "by count, actions": [0, 0, 0]}
        for tile in pick:
            seqs = []
            for i in range(tile * 256, tile * 256 + 256):
                t = np.ascontiguousarray(tups[i], dtype=np.uint64)
                n = lib.kc_spec_successors(C.byref(c), t.ctypes.data_as(C.POINTER(C.c_uint64)), acts, out, 64,
                                           C.byref(fa))
                seqs.append(tuple(acts[k] for k in range(max(n, 0))))
            orders = {
                "lane=parent": seqs,
                "by count": sorted(seqs, key=lambda s: -len(s)),
                "by count, actions": sorted(seqs, key=lambda s: (-len(s), s)),
            }
            for name, o in orders.items():
                for w in range(4):
                    a, b, l = wave_cost(o[64 * w:64 * w + 64])
                    tot[name][0] += a
                    tot[name][1] += b
                    tot[name][2] += l
        row = {"level": L, "width": int(len(tups)), "tiles": int(len(pick))}
        for name, (trips, bodies, lanes) in tot.items():
            row[name] = {"wave_trips": trips, "bodies": bodies, "bodies_per_trip": round(bodies / max(trips, 1), 2),
                         "busy": round(lanes / max(64 * trips, 1), 3)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
