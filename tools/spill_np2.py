"""NP=2 with the seen-set capped (seen-set spill): wall time, the spill's
statistics and its host-time breakdown, exact counts checked against
tests/golden/np2_full.json.

  python tools/spill_np2.py [hbm_gib] [host_gib] [spill_dir]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))
import torch  # noqa: E402,F401

from kubecheck import ModelChecker, ModelConfig  # noqa: E402

hbm = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
host = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
sdir = sys.argv[3] if len(sys.argv) > 3 else None
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "np2_full.json")))
cfg = ModelConfig(np=2, keep_trace=False, seen_hbm_bytes=int(hbm * (1 << 30)),
                  seen_host_bytes=int(host * (1 << 30)), spill_dir=sdir, verbose=1)
with ModelChecker(cfg) as mc:
    t0 = time.perf_counter()
    r = mc.run()
    dt = time.perf_counter() - t0
ok = (r.distinct, r.generated, r.depth, r.level_width) == (fx["distinct"], fx["generated"], fx["depth"],
                                                           fx["level_width"])
print(json.dumps({"seen_hbm_gib": hbm, "seen_host_gib": host, "spill_dir": sdir, "seconds": round(dt, 3),
                  "distinct_per_s": round(r.distinct / dt, 1), "exact": ok, "seen": r.seen,
                  "cand_buffer_peak_bytes": r.cand_buffer_peak_bytes,
                  "cand_overflow_records": r.cand_overflow_records}), flush=True)
if not ok:
    sys.exit(1)
