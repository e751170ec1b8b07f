"""Owner-function study for the sharded path: for candidate
projections of the packed state that feed the fingerprint's owner bits,
the fraction of successors that change owner (records the all-to-all must
carry) and the per-level balance (max/mean states per rank; a level takes as
long as its busiest rank), at R = 2, 4, 8, on levels of the NP=2 model
captured by the GPU engine (sampled).  Host-side arithmetic mirrors
kubeapi_spec.h owner_hash (4 owner bits; owner = floor(bits * R / 16)).

  python tools/owner_balance.py [levels...]"""
import collections
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

M64 = (1 << 64) - 1


def ohash(w0, wo):
    z = (w0 * 0x9e3779b97f4a7c15 + wo) & M64
    z ^= z >> 31
    z = (z * 0xbf58476d1ce4e5b9) & M64
    return z >> 60


def fold(*ws):
    h = 0
    for w in ws:
        h = ((h ^ w) * 0xff51afd7ed558ccd) & M64
        h ^= h >> 33
    return h


# NP=2 packed words: 0 apiState, 1 client, 2 PVC controller 1, 3 PVC controller 2, 4-5 listRequests objs
def rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


PROJ = {
    "w0,pvc1 (round 2)": lambda w: ohash(w[0], w[2]),
    "w0,objs (round 3, kubeapi_spec.h owner_proj)": lambda w: ohash(w[0], rotl(w[4], 7) ^ rotl(w[5], 24)),
    "w0,objs": lambda w: ohash(w[0], fold(w[4], w[5])),
    "w0,objs,rq": lambda w: ohash(w[0], fold(w[4], w[5], (w[1] >> 5) & 0x3f, (w[2] >> 5) & 0x3f, (w[3] >> 5) & 0x3f)),
}


def main():
    levels = [int(x) for x in sys.argv[1:]] or [40, 60, 86, 110, 140, 165]
    lib = kubecheck.load()
    cfg = ModelConfig(np=2)
    c = cfg.to_c()
    W = lib.kc_spec_state_words(1, 2, 1)
    rng = np.random.RandomState(7)
    acts = (C.c_int * 64)()
    fa = C.c_int()

    def pack(t):
        t = np.ascontiguousarray(t, dtype=np.uint64)
        w = (C.c_uint64 * W)()
        lib.kc_spec_pack(C.byref(c), t.ctypes.data_as(C.POINTER(C.c_uint64)), w)
        return [int(x) for x in w]

    for L in levels:
        with ModelChecker(ModelConfig(np=2, max_levels=L + 1, keep_trace=False)) as mc:
            mc.capture_level(L)
            mc.run()
            tups = mc.level_tuples(L)
        tw = tups.shape[1]
        out = (C.c_uint64 * (64 * tw))()
        bal_idx = rng.choice(len(tups), min(len(tups), 100000), replace=False)
        packed = [pack(tups[i]) for i in bal_idx]
        pairs = []
        for i in bal_idx[:8000]:
            t = np.ascontiguousarray(tups[i], dtype=np.uint64)
            pw = pack(t)
            n = lib.kc_spec_successors(C.byref(c), t.ctypes.data_as(C.POINTER(C.c_uint64)), acts, out, 64, C.byref(fa))
            for k in range(max(n, 0)):
                pairs.append((pw, pack(np.frombuffer(out, dtype=np.uint64, count=tw, offset=k * tw * 8))))
        row = {"level": L, "width": int(len(tups)), "sampled_states": len(packed), "sampled_successors": len(pairs)}
        for name, f in PROJ.items():
            cls = [f(w) for w in packed]
            pc = [(f(p), f(q)) for p, q in pairs]
            for R in (2, 4, 8):
                cnt = collections.Counter(x * R // 16 for x in cls)
                row[f"{name} R{R} balance"] = round(max(cnt.values()) / (len(cls) / R), 3)
                row[f"{name} R{R} remote"] = round(sum(a * R // 16 != b * R // 16 for a, b in pc) / max(len(pc), 1), 3)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
