#!/usr/bin/env python3
"""Diagnostic: R shards (kc_shard_*) emulated in one process on one GPU, the
exchange done by slicing the device send buffers (as tests/test_gpu_shard.py),
over a whole model.  Prints totals and the time of each stage summed over the
shards, i.e. the kernel work an R-GPU run spreads over R devices.

  python tools/exp_emulate.py --R 2 --np 2
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import torch  # noqa: E402
from kubecheck import ModelConfig  # noqa: E402
from kubecheck.distributed import HipShard, NONE_KEY  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--R", type=int, default=2)
ap.add_argument("--np", type=int, default=2)
ap.add_argument("--nc", type=int, default=1)
ap.add_argument("--runs", type=int, default=1)
a = ap.parse_args()

cfg = ModelConfig(nc=a.nc, np=a.np, fpset_slots=1 << 20)
shards = [HipShard(cfg, r, a.R) for r in range(a.R)]
rb = shards[0].record_bytes
rw = rb // 8
for run in range(a.runs):
    prof = {"expand": 0.0, "pack": 0.0, "exchange": 0.0, "insert": 0.0}
    t0 = time.perf_counter()
    n = sum(s.init() for s in shards)
    widths, err, records = [n], NONE_KEY, 0
    while True:
        sends, counts = [], []
        for s in shards:
            t = time.perf_counter()
            c, e = s.expand()
            prof["expand"] += time.perf_counter() - t
            err = min(err, e)
            buf = torch.empty(max(sum(c), 1) * rw, dtype=torch.int64, device="cuda")
            t = time.perf_counter()
            s.pack(buf)
            prof["pack"] += time.perf_counter() - t
            sends.append(buf)
            counts.append(c)
            records += sum(c)
        total = 0
        for r, s in enumerate(shards):
            t = time.perf_counter()
            parts, m = [], 0
            for src in range(a.R):
                off = sum(counts[src][:r]) * rw
                parts.append(sends[src][off: off + counts[src][r] * rw])
                m += counts[src][r]
            recv = torch.cat(parts) if m else torch.empty(rw, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            prof["exchange"] += time.perf_counter() - t
            t = time.perf_counter()
            nn, e = s.insert(recv, m)
            prof["insert"] += time.perf_counter() - t
            err = min(err, e)
            total += nn
        del sends, parts, recv
        if err != NONE_KEY or total == 0:
            break
        for s in shards:
            s.advance()
        widths.append(total)
    dt = time.perf_counter() - t0
    res = [s.result() for s in shards]
    distinct = sum(r["distinct"] for r in res)
    gen = sum(r["init"] + r["generated"] for r in res)
    print({"R": a.R, "distinct": distinct, "generated": gen, "depth": len(widths),
           "err": err if err != NONE_KEY else None, "records": records,
           "per_shard_distinct": [r["distinct"] for r in res], "seconds": round(dt, 3)}, flush=True)
    print({k: round(v * 1e3, 1) for k, v in prof.items()}, "ms (summed over shards)", flush=True)
for s in shards:
    s.close()
