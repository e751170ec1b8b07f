#!/usr/bin/env python3
"""Diagnostic: the sharded driver (kubecheck.distributed) on this process's
GPU at world size 1 (RCCL), printing the result summary.

  python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/exp_sharded.py [--np 2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from kubecheck import ModelConfig  # noqa: E402
from kubecheck.distributed import HipShard, ShardedModelChecker  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--np", type=int, default=2)
ap.add_argument("--nc", type=int, default=1)
ap.add_argument("--runs", type=int, default=2)
a = ap.parse_args()
for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0"), ("MASTER_ADDR", "127.0.0.1"),
             ("MASTER_PORT", "29533")):
    os.environ.setdefault(k, v)                     # world 1 without torchrun
local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
cfg = ModelConfig(nc=a.nc, np=a.np, device=local, fpset_slots=1 << 20)
mc = ShardedModelChecker(cfg, HipShard(cfg, dist.get_rank(), dist.get_world_size()))
for _ in range(a.runs):
    r = mc.run()
    if dist.get_rank() == 0:
        print({k: r[k] for k in ("distinct", "generated", "depth", "error", "complete", "seconds")},
              r.get("error_action"), r.get("error_invariant"), r.get("error_level"), r["level_width"][-5:],
              flush=True)
        if getattr(mc, "_prof", None):
            print({k: round(v * 1e3, 1) for k, v in mc._prof.items()}, "ms", flush=True)
dist.destroy_process_group()
