"""Model_1 through the native sharded loop at world 1 (the narrow levels,
shard_narrow.h), for a rocprofv3 kernel trace of the per-level launches.
  rocprofv3 --kernel-trace --stats -- python3 tools/sn_trace.py [--force]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))
if "--force" in sys.argv:
    os.environ["KC_RCCL_FORCE"] = "1"

import torch  # noqa: E402,F401

from kubecheck import ModelConfig  # noqa: E402
from kubecheck.distributed import NativeShardedChecker  # noqa: E402

mc = NativeShardedChecker(ModelConfig(keep_trace=False), 0, 1)
try:
    for _ in range(5):
        r = mc.run()
    print(r["distinct"], r["depth"], r["narrow_levels"])
finally:
    mc.close()
