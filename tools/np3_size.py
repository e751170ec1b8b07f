"""Sizing NP=3 (SURVEY §8(d) config 2 secondary) on the GPU: level widths
and distinct states of a growing prefix, from one run per prefix length,
with the per-level growth ratio (the model is far larger than NP=2: the
oracle's first 40 levels already hold 50.8M states, +33% per level).

  python tools/np3_size.py 50 55 60"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))
import torch  # noqa: E402,F401

from kubecheck import ModelChecker, ModelConfig  # noqa: E402

for L in map(int, sys.argv[1:] or ["50"]):
    t0 = time.perf_counter()
    with ModelChecker(ModelConfig(np=3, max_levels=L, keep_trace=False)) as mc:
        r = mc.run()
    w = r.level_width
    print(json.dumps({"levels": L, "distinct": r.distinct, "generated": r.generated, "seconds": round(
        time.perf_counter() - t0, 2), "last_widths": w[-5:], "growth": [round(w[i] / w[i - 1], 4) for i in
                                                                         range(len(w) - 5, len(w))],
        "level_width": w}), flush=True)
