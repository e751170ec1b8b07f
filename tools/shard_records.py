"""Records the sharded NP=2 check sends between ranks (the all-to-all's
volume) and its time, with R ranks emulated on one GPU (kc_group_create_local):
what the owner function costs in xGMI bytes.

  python tools/shard_records.py [R ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import torch  # noqa: E402,F401

from kubecheck import ModelConfig  # noqa: E402
from kubecheck.distributed import NativeShardedChecker  # noqa: E402


def main():
    for R in [int(x) for x in sys.argv[1:]] or [2, 4, 8]:
        mc = NativeShardedChecker(ModelConfig(np=2, keep_trace=False), emulate=R)
        try:
            mc.run()
            t0 = time.perf_counter()
            r = mc.run()
            dt = time.perf_counter() - t0
            print(json.dumps({"R": R, "ms": round(dt * 1e3, 1), "distinct": r["distinct"], "generated": r["generated"],
                              "records_sent": mc.records_sent, "record_bytes": mc.record_bytes,
                              "bytes_sent": mc.records_sent * mc.record_bytes}), flush=True)
        finally:
            mc.close()


if __name__ == "__main__":
    main()
