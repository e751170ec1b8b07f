"""Fingerprint-owner-sharded FPSet across GPUs (one process per GPU).

The multi-GPU form of the tlc2.tool.fp.FPSet seam (the reference run used
one OffHeapDiskFPSet, MC.out:5; TLC's own MultiFPSet splits by the top bits
of the fingerprint [ext-TLC]).  Rank r owns the fingerprints with
owner(fp) = floor(fp * R / 2^63) and their HBM table.  Every rank produces
fingerprints for every owner (as TLC workers do), so each batch is:

    partition by owner (kc_fpset_partition_dev, stable counting sort)
      -> all-to-all of the per-owner counts (R int64)
      -> all-to-all of the fingerprints over RCCL (xGMI), device to device
      -> insert / look up the received fps in the local table

This module drives BASELINE.json configs[3]:
1e10 fingerprints of the perm63 stress stream (kc_stress_fps_dev; every
input distinct, so the final size is exactly n) inserted by R ranks, then
as many lookups, half present.  Strong scaling: the 1e10 total is split
over the ranks.

The stage implementation ("backend") is :class:`HipFPSetShard` on the GPU;
the CPU tests drive the same code under gloo with a numpy emulation.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

from . import FPSet, stress_fps_dev

STRESS_SEED = 0x5EED0000


class HipFPSetShard:
    """This rank's FPSet table and stages on its GPU."""

    device_type = "cuda"

    def __init__(self, capacity: int, device: int = 0):
        self.fs = FPSet(capacity=capacity, device=device)

    def gen(self, seed: int, kind: int, n_ins: int, start: int, n: int, out, stream=None) -> None:
        stress_fps_dev(seed, kind, n_ins, start, n, out, stream)

    def partition(self, fps, n: int, world: int, out, stream=None) -> List[int]:
        return self.fs.partition_dev(fps, n, world, out, stream)

    def insert(self, fps, n: int, stream=None) -> int:
        return self.fs.insert_count_dev(fps, n, stream)

    def lookup(self, fps, n: int, stream=None) -> int:
        return self.fs.contains_count_dev(fps, n, stream)

    def size(self) -> int:
        return self.fs.size()

    def table_bytes(self) -> int:
        return self.fs.capacity() * 8

    def close(self) -> None:
        self.fs.close()


def rank_range(n: int, rank: int, world: int):
    """[lo, hi) of a length-n stream that rank `rank` produces."""
    return n * rank // world, n * (rank + 1) // world


class ShardedFPSetStress:
    """Batched, owner-routed insert/lookup stress over torch.distributed."""

    def __init__(self, backend, group=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.be, self.group = torch, dist, backend, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 16:
            raise ValueError("sharded FPSet: at most 16 ranks (kc_fpset_partition_dev)")
        self.dev = torch.device("cuda", torch.cuda.current_device()) \
            if backend.device_type == "cuda" else torch.device("cpu")
        self.stream = torch.cuda.current_stream() if self.dev.type == "cuda" else None
        self._bufs: Dict[str, object] = {}
        self.sent = 0                 # fingerprints this rank sent to other ranks

    def _buf(self, name: str, n: int):
        b = self._bufs.get(name)
        if b is None or b.numel() < n:
            b = self.torch.empty(max(n, 1), dtype=self.torch.int64, device=self.dev)
            self._bufs[name] = b
        return b

    def _phase(self, seed: int, kind: int, n_ins: int, n_total: int, batch: int) -> int:
        """Produce this rank's share of a stream in batches, route every fp
        to its owner, insert (kind 0) or look up (kind 1) there.  Returns
        this rank's count of new (kind 0) or found (kind 1) fps."""
        torch, dist, R, st = self.torch, self.dist, self.world, self.stream
        lo, hi = rank_range(n_total, self.rank, R)
        rounds = -(-max(rank_range(n_total, r, R)[1] - rank_range(n_total, r, R)[0]
                        for r in range(R)) // batch)
        gen = self._buf("gen", batch)
        part = self._buf("part", batch)
        total = 0
        for k in range(rounds):
            start = lo + k * batch
            m = max(0, min(batch, hi - start))
            self.be.gen(seed, kind, n_ins, start, m, gen, st)
            if R == 1:
                recv, nrecv = gen, m
            else:
                counts = self.be.partition(gen, m, R, part, st)
                cin = torch.tensor(counts, dtype=torch.int64, device=self.dev)
                cout = torch.empty(R, dtype=torch.int64, device=self.dev)
                dist.all_to_all_single(cout, cin, group=self.group)
                rcounts = cout.tolist()
                nrecv = sum(rcounts)
                recv = self._buf("recv", nrecv)
                dist.all_to_all_single(recv[:nrecv], part[:m], output_split_sizes=rcounts,
                                       input_split_sizes=counts, group=self.group)
                self.sent += m - counts[self.rank]
            total += self.be.insert(recv, nrecv, st) if kind == 0 else self.be.lookup(recv, nrecv, st)
        return total

    def _sync(self):
        if self.dev.type == "cuda":
            self.torch.cuda.synchronize()
        self.dist.barrier(group=self.group)

    def _max(self, x: float) -> float:
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def _sum(self, vals: List[int]) -> List[int]:
        t = self.torch.tensor(vals, dtype=self.torch.int64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return [int(x) for x in t.tolist()]

    def run(self, n: int, batch: int, n_lookup: int, seed: int = STRESS_SEED) -> dict:
        """Insert stream [0, n) then lookups [0, n_lookup); totals over all
        ranks.  Times are max over ranks, barrier-bracketed."""
        self.sent = 0
        self._sync()
        t0 = time.perf_counter()
        new = self._phase(seed, 0, n, n, batch)
        self._sync()
        t1 = time.perf_counter()
        found = self._phase(seed, 1, n, n_lookup, batch) if n_lookup else 0
        self._sync()
        t2 = time.perf_counter()
        ti, tl = self._max(t1 - t0), self._max(t2 - t1)
        new_all, found_all, size_all, sent_all = self._sum([new, found, self.be.size(), self.sent])
        return {"inserted_new": new_all, "found": found_all, "size": size_all,
                "local_size": self.be.size(), "insert_seconds": ti, "lookup_seconds": tl,
                "fps_sent": sent_all, "world": self.world}


def capacity_for(n: int, world: int, load: float) -> int:
    """kc_fpset_create capacity for one rank's table so that its share of n
    uniform fps (n/R + 8 sigma) lands at `load` (slots = capacity * 4/3)."""
    share = n / world
    share += 8 * share ** 0.5 + 64
    return int(share / load * 3 / 4)


def bench_sharded_fpset(args) -> Optional[dict]:
    """bench.py --workload fpset --gpus N (N processes, one per GPU)."""
    import os

    import torch
    import torch.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rank, world = dist.get_rank(), dist.get_world_size()
    n = int(args.fp_count)
    batch = 1 << 24
    res = None
    for step in range(args.warmup + args.steps):
        be = HipFPSetShard(capacity_for(n, world, args.fp_load), device=local)
        drv = ShardedFPSetStress(be)
        r = drv.run(n, batch, n)
        table_bytes = be.table_bytes()
        be.close()
        if r["size"] != n or r["inserted_new"] != n or r["found"] != (n + 1) // 2:
            raise RuntimeError(f"sharded fpset stress: size {r['size']} new {r['inserted_new']} "
                               f"found {r['found']} for n={n}")
        if step >= args.warmup:
            if res is None:
                res = dict(r, insert_seconds=0.0, lookup_seconds=0.0)
            res["insert_seconds"] += r["insert_seconds"]
            res["lookup_seconds"] += r["lookup_seconds"]
    dist.destroy_process_group()
    if rank != 0:
        return None
    tin, tlk = res["insert_seconds"], res["lookup_seconds"]
    gbs = n * args.steps * 64 / tin / 1e9
    return {
        "metric": "FPSet probe HBM GB/s (insert)", "value": round(gbs, 1), "unit": "GB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(tin * 1e3 / args.steps, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic perm63 fingerprint stream generated on device",
        "config": {"workload": f"FPSet stress sharded over {world} GPUs: {n} inserts + {n} lookups "
                               f"to {args.fp_load:.0%} load, batch {batch} per rank",
                   "path": "sharded FPSet (owner partition + RCCL all-to-all per batch)",
                   "table_bytes_per_gpu": table_bytes,
                   "inserts_per_s": round(n * args.steps / tin, 1),
                   "lookups_per_s": round(n * args.steps / tlk, 1),
                   "fps_sent_per_step": res["fps_sent"],
                   "xgmi_bytes_per_step": res["fps_sent"] * 8,
                   "lookups_found": res["found"]},
        "roofline": {"bound": "hbm", "achieved": round(gbs / world, 2), "peak": 8000.0,
                     "unit": "GB/s", "frac": round(gbs / world / 8000.0, 4), "traffic": None,
                     "kernel": "k_insert_count", "per": "GPU (achieved = whole-job GB/s / N)"},
    }
