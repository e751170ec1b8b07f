"""One rank of tests/test_gpu_hostcomm.py: the native sharded level loop
(kc_group_run) with one shard per process and the collectives over gloo
(kc_group_create_host, kubecheck.distributed.GlooHostComm).  Every rank
uses device 0.  Launched by torch.distributed.run; argv[1] = path of a JSON
list of cases {"name", "kw", "env"}; rank 0 prints one JSON line per case
(every rank does for cases with "all_ranks")."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import torch  # noqa: E402,F401
import torch.distributed as dist  # noqa: E402

from kubecheck import ModelConfig  # noqa: E402
from kubecheck.distributed import NativeShardedChecker  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    cases = json.load(open(sys.argv[1]))
    for case in cases:
        saved = {k: os.environ.get(k) for k in case.get("env", {})}
        os.environ.update(case.get("env", {}))
        out = {"case": case["name"], "rank": rank, "world": world}
        mc = None
        try:
            mc = NativeShardedChecker(ModelConfig(device=0, **case["kw"]), rank, world, transport="host")
            r = mc.run()
            out.update(r)
            out["records_sent"] = mc.records_sent
        except Exception as e:          # noqa: BLE001  (the fault cases expect one on every rank)
            out["exception"] = str(e)
        finally:
            if mc is not None:
                mc.close()
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        if rank == 0 or case.get("all_ranks"):
            # one write of the whole line (the ranks share the launcher's stdout)
            os.write(1, ("RESULT " + json.dumps(out) + "\n").encode())
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
