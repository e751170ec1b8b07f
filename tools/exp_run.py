#!/usr/bin/env python3
"""Diagnostic: run one model check (default NP=2) a few times and print the
per-kernel HIP-event times; with KC_ABLATE=1 the engine also times cut-down
k_claim variants (successors + LDS dedup, successors only) on scratch buffers.

  KC_ABLATE=1 python tools/exp_run.py [--np 2] [--runs 2]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import torch  # noqa: F401,E402
import kubecheck  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nc", type=int, default=1)
ap.add_argument("--np", type=int, default=2)
ap.add_argument("--runs", type=int, default=2)
ap.add_argument("--slots", type=int, default=20, help="log2 initial seen-set slots")
a = ap.parse_args()
cfg = kubecheck.ModelConfig(nc=a.nc, np=a.np, keep_trace=True, timing=True, fpset_slots=1 << a.slots)
with kubecheck.ModelChecker(cfg) as mc:
    for k in range(a.runs):
        t0 = time.perf_counter()
        r = mc.run()
        dt = time.perf_counter() - t0
        kt = mc.kernel_times()
        print(f"run {k}: {dt * 1e3:.1f} ms distinct {r.distinct} generated {r.generated} depth {r.depth} "
              f"probes {r.fpset_probes} settles {r.batch_inserts} "
              + " ".join(f"{n}={v[0]:.1f}ms" for n, v in kt.items()), flush=True)
