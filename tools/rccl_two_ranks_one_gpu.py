"""Probe: can the native sharded loop's RcclComm run two ranks (two processes)
on ONE GPU?  The driver's `bench.py --gpus N` is the first place RcclComm
runs at world > 1; if RCCL accepts two ranks on one device, this exercises
its all-gather, the grouped send/recv exchange plan and the broadcast at
world 2 before that.

  python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
      --master-addr=127.0.0.1 --master-port=29577 tools/rccl_two_ranks_one_gpu.py [--np2] [--trace]

Every rank uses device 0; the RCCL unique id travels over a gloo group.
Rank 0 prints one JSON line per check."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import torch  # noqa: E402,F401
import torch.distributed as dist  # noqa: E402

from kubecheck import ModelConfig  # noqa: E402
from kubecheck.distributed import NativeShardedChecker  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    g = os.path.join(ROOT, "tests", "golden")
    cases = [("model1", {}, json.load(open(os.path.join(g, "model1_mcout.json"))))]
    if "--np2" in sys.argv:
        cases.append(("np2", dict(np=2, keep_trace=False), json.load(open(os.path.join(g, "np2_full.json")))))
    if "--trace" in sys.argv:
        # the NC=2 C4 assertion race (BASELINE configs[4]): error walk over ranks (broadcast)
        cases.append(("nc2_np0", dict(nc=2, np=0), None))
    for name, kw, want in cases:
        mc = NativeShardedChecker(ModelConfig(device=0, **kw), rank, world)
        try:
            mc.run()
            t0 = time.perf_counter()
            r = mc.run()
            dt = time.perf_counter() - t0
        finally:
            mc.close()
        if rank == 0:
            out = {"case": name, "world": world, "ms": round(dt * 1e3, 3), "distinct": r["distinct"],
                   "generated": r["generated"], "depth": r["depth"], "error": r["error"],
                   "trace_len": r.get("trace_len"), "records_sent": mc.records_sent}
            if want is not None:
                out["exact"] = (r["distinct"], r["generated"], r["depth"]) == \
                    (want["distinct"], want["generated"], want["depth"])
            print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
