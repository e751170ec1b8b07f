"""Fingerprint-owner-sharded BFS across GPUs (one process per GPU).

Replaces TLC's single-host worker pool for the KubeAPI hot path (TLC's own
distributed mode, RMI TLCServer/TLCWorker, is off in Model_1:
KubeAPI___Model_1.launch:4-7).  Each rank owns the fingerprints with
owner(fp) = floor(fp * R / 2^63), their FPSet shard and the frontier of the
states it owns.  Per BFS level:

    expand (local dedup)  ->  pack records per owner  ->  all-to-all (counts,
    then records)  ->  insert (dedup by min key, FPSet shard, compact)  ->
    all-reduce (new-state count SUM, error key MIN)  ->  advance

All state data moves over RCCL (torch.distributed backend "nccl" on ROCm)
between HBM buffers; the host only sees counts.  Level-synchronous, so
traces stay shortest and totals do not depend on R.

The stage implementation ("backend") is libkubecheck.so's kc_shard_* on the
GPU (:class:`HipShard`).  The driver only needs the stage protocol, which
is how the CPU tests exercise it under gloo with a host emulation of the
stages.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import re
import time
from typing import List, Optional, Sequence

import numpy as np

from . import ACTIONS, CLAIM_MODES, INVARIANTS, ModelConfig, Spec
from ._lib import (HC_ALL_GATHER, HC_ALL_REDUCE, HC_BROADCAST, HC_EXCHANGE, KcHostComm, KcResult, check,
                   load)

NONE_KEY = (1 << 64) - 1       # "no error" (the library's ~0)
M44 = (1 << 44) - 1
MAX_WORLD = 15                 # keys carry the rank in 4 bits (shard.hip); 15 = Init-state keys


def key_to_i64(key: int) -> int:
    """Order-preserving map of an unsigned 64-bit key into int64 (for the
    int64 collectives): key - 2^63, so NONE_KEY becomes INT64_MAX and keys
    of ranks >= 8 (>= 2^63) stay ordered below it."""
    return int(key) - (1 << 63)


def i64_to_key(v: int) -> int:
    return int(v) + (1 << 63)


def owner(fp: int, world: int) -> int:
    """owner(fp) = floor(fp * R / 2^63) for a normalised fingerprint."""
    return ((fp & ((1 << 63) - 1)) * world) >> 63


class HipShard:
    """kc_shard_* stages on this process's GPU (device = cfg.device)."""

    device_type = "cuda"

    def __init__(self, cfg: ModelConfig, rank: int, world: int):
        self._lib = load()
        self.cfg, self.rank, self.world = cfg, rank, world
        self._c = cfg.to_c()
        self._h = C.c_void_p()
        check("kc_shard_create", self._lib.kc_shard_create(C.byref(self._c), rank, world, C.byref(self._h)))
        self.record_bytes = int(self._lib.kc_shard_record_bytes(self._h))
        self.tuple_words = self._lib.kc_spec_tuple_words(cfg.nc, cfg.np, cfg.ns)
        self.stream_ordered = False

    def use_stream(self, stream) -> None:
        """Run the stages on `stream` (a torch.cuda.Stream), the one the
        driver's RCCL collectives use: no host sync between pack, the
        all-to-all and insert."""
        check("kc_shard_set_stream", self._lib.kc_shard_set_stream(self._h, C.c_void_p(stream.cuda_stream)))
        self.stream_ordered = True

    def init(self) -> int:
        n = C.c_uint64()
        check("kc_shard_init", self._lib.kc_shard_init(self._h, C.byref(n)))
        return n.value

    def init_error(self) -> int:
        """Key of this rank's first Init state violating an invariant (~0: none)."""
        k = C.c_uint64()
        check("kc_shard_init_error", self._lib.kc_shard_init_error(self._h, C.byref(k)))
        return k.value

    def expand(self):
        counts = (C.c_uint64 * self.world)()
        err = C.c_uint64()
        check("kc_shard_expand", self._lib.kc_shard_expand(self._h, counts, C.byref(err)))
        return [int(x) for x in counts], int(err.value)

    def pack(self, send) -> None:
        check("kc_shard_pack", self._lib.kc_shard_pack(self._h, C.c_void_p(send.data_ptr())))

    def insert(self, recv, n: int):
        nn, err = C.c_uint64(), C.c_uint64()
        check("kc_shard_insert", self._lib.kc_shard_insert(
            self._h, C.c_void_p(recv.data_ptr()), n, C.byref(nn), C.byref(err)))
        return int(nn.value), int(err.value)

    def advance(self) -> None:
        check("kc_shard_advance", self._lib.kc_shard_advance(self._h))

    def parent_key(self, level: int, idx: int) -> int:
        k = C.c_uint64()
        check("kc_shard_parent_key", self._lib.kc_shard_parent_key(self._h, level, idx, C.byref(k)))
        return int(k.value)

    def result(self) -> dict:
        r = KcResult()
        check("kc_shard_result", self._lib.kc_shard_result(self._h, C.byref(r)))
        return {"act_gen": [int(r.act_gen[i]) for i in range(len(ACTIONS))],
                "act_dist": [int(r.act_dist[i]) for i in range(len(ACTIONS))],
                "init": int(r.init), "generated": int(r.generated), "distinct": int(r.distinct),
                "fpset_slots": int(r.fpset_slots), "deferred": int(r.deferred_states)}

    def claim_times(self):
        """(k_claim ms, launches, parents) since the last call."""
        ms, n, p = C.c_double(), C.c_uint64(), C.c_uint64()
        check("kc_shard_claim_times", self._lib.kc_shard_claim_times(self._h, C.byref(ms), C.byref(n),
                                                                      C.byref(p)))
        return ms.value, int(n.value), int(p.value)

    def close(self) -> None:
        if self._h:
            self._lib.kc_shard_destroy(self._h)
            self._h = C.c_void_p()


class GlooHostComm:
    """kc_host_comm over a torch.distributed process group on host tensors
    (gloo): the native level loop with one shard per process and a transport
    other than RCCL (kc_group_create_host).  Several ranks may then share one
    GPU, which RCCL refuses ("duplicate GPU"); the tests use it to run the
    one-shard-per-process loop at world > 1 on the one-GPU box.  Callbacks
    run on the thread inside kc_group_run; an exception becomes rc -1 (the
    loop then fails with -EIO) and is kept in `.errors`."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self._t, self._d, self.group = torch, dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.errors: List[str] = []
        self.ops = KcHostComm(None, HC_ALL_GATHER(self._guard(self._all_gather)),
                              HC_EXCHANGE(self._guard(self._exchange)),
                              HC_BROADCAST(self._guard(self._broadcast)),
                              HC_ALL_REDUCE(self._guard(self._all_reduce)))

    def _guard(self, fn):
        def call(*a):
            try:
                fn(*a)
                return 0
            except Exception as e:          # noqa: BLE001  (crosses the C-ABI as rc -1)
                self.errors.append(f"{fn.__name__}: {e!r}")
                return -1
        return call

    def _words(self, ptr, n):
        return self._t.from_numpy(np.ctypeslib.as_array(ptr, (int(n),)).view(np.int64))

    def _all_gather(self, _ctx, inp, n, out):
        src = self._words(inp, n).clone()
        parts = [self._t.empty(int(n), dtype=self._t.int64) for _ in range(self.world)]
        self._d.all_gather(parts, src, group=self.group)
        self._words(out, n * self.world).copy_(self._t.cat(parts))

    def _exchange(self, _ctx, xf, nx, sendbuf, recvbuf):
        x = np.ctypeslib.as_array(xf, (int(nx), 4)).astype(np.int64) if nx else np.zeros((0, 4), np.int64)
        sends, recvs = x[x[:, 1] == 1], x[x[:, 1] == 0]
        span = lambda v: int((v[:, 2] + v[:, 3]).max()) if len(v) else 0   # noqa: E731
        sb = np.ctypeslib.as_array((C.c_uint8 * max(span(sends), 1)).from_address(sendbuf)) if len(sends) else None
        rb = np.ctypeslib.as_array((C.c_uint8 * max(span(recvs), 1)).from_address(recvbuf)) if len(recvs) else None
        reqs, piece = [], {}
        own_s, own_r = [], []
        for peer, snd, off, nb in x.tolist():
            if peer == self.rank:                      # (never planned today: own claims stay in place)
                (own_s if snd else own_r).append((off, nb))
                continue
            k = piece.get((peer, snd), 0)              # k-th piece of this (peer, direction): tag k
            piece[(peer, snd)] = k + 1
            if snd:
                reqs.append(self._d.isend(self._t.from_numpy(sb[off: off + nb]), peer, group=self.group, tag=k))
            else:
                reqs.append(self._d.irecv(self._t.from_numpy(rb[off: off + nb]), peer, group=self.group, tag=k))
        for (so, nb), (ro, _) in zip(own_s, own_r):
            rb[ro: ro + nb] = sb[so: so + nb]
        for r in reqs:
            r.wait()

    def _broadcast(self, _ctx, root, v):
        t = self._words(v, 1).clone()
        self._d.broadcast(t, src=int(root), group=self.group)
        self._words(v, 1).copy_(t)

    def _all_reduce(self, _ctx, v, n):
        t = self._words(v, n).clone()
        self._d.all_reduce(t, group=self.group)
        self._words(v, n).copy_(t)


class NativeShardedChecker:
    """The sharded BFS with the native level loop (libkubecheck kc_group_*):
    the same protocol and result dict as :class:`ShardedModelChecker`, with
    the levels driven in C++ over RCCL instead of from Python.

    * ``NativeShardedChecker(cfg, rank, world)`` inside a torch.distributed
      job (one process per GPU): rank 0 makes the RCCL id, torch broadcasts
      it, every rank joins one RCCL communicator.
    * ``NativeShardedChecker(cfg, emulate=R)``: ranks 0..R-1 in this process
      on one GPU, collectives by device copies (the multi-rank protocol on
      one GPU).
    * ``transport="host"``: one shard per process as with RCCL, the
      collectives over the torch.distributed group on host buffers
      (:class:`GlooHostComm`, kc_group_create_host)."""

    def __init__(self, cfg: ModelConfig, rank: int = 0, world: int = 1, emulate: int = 0, group=None,
                 transport: str = "rccl"):
        self._lib = load()
        self.cfg = cfg
        self._c = cfg.to_c()
        self.spec = Spec(cfg)
        self._shards = []
        self._g = C.c_void_p()
        if emulate:
            for r in range(emulate):
                h = C.c_void_p()
                check("kc_shard_create", self._lib.kc_shard_create(C.byref(self._c), r, emulate, C.byref(h)))
                self._shards.append(h)
            arr = (C.c_void_p * emulate)(*[h.value for h in self._shards])
            check("kc_group_create_local", self._lib.kc_group_create_local(arr, emulate, C.byref(self._g)))
            self.world = emulate
        else:
            import torch
            import torch.distributed as dist

            h = C.c_void_p()
            check("kc_shard_create", self._lib.kc_shard_create(C.byref(self._c), rank, world, C.byref(h)))
            self._shards.append(h)
            self.world = world
            if transport == "host":
                self.host_comm = GlooHostComm(group)
                check("kc_group_create_host",
                      self._lib.kc_group_create_host(h, C.byref(self.host_comm.ops), C.byref(self._g)))
                self.records_sent = 0
                self.record_bytes = int(self._lib.kc_shard_record_bytes(self._shards[0]))
                return
            uid = C.create_string_buffer(128)
            if rank == 0:
                check("kc_rccl_unique_id", self._lib.kc_rccl_unique_id(uid))
            if world > 1:
                t = torch.frombuffer(bytearray(uid.raw), dtype=torch.uint8).to(
                    "cuda" if dist.get_backend(group) == "nccl" else "cpu")
                dist.broadcast(t, src=0, group=group)
                uid = C.create_string_buffer(bytes(t.cpu().tolist()), 128)
            check("kc_group_create_rccl", self._lib.kc_group_create_rccl(h, uid, C.byref(self._g)))
            self.world = world
        self.records_sent = 0
        self.record_bytes = int(self._lib.kc_shard_record_bytes(self._shards[0]))

    def run(self) -> dict:
        r = KcResult()
        rc = self._lib.kc_group_run(self._g, C.byref(r))
        hc = getattr(self, "host_comm", None)
        if rc < 0 and hc is not None and hc.errors:
            raise RuntimeError(f"kc_group_run: host transport failed: {hc.errors[0]}")
        check("kc_group_run", rc)
        self.records_sent = int(self._lib.kc_group_records_sent(self._g))
        na = len(ACTIONS)
        out = {
            "init": int(r.init), "generated": int(r.generated), "distinct": int(r.distinct),
            "depth": int(r.depth), "level_width": [int(r.level_width[i]) for i in range(r.nlevels)],
            "act_gen": {a: int(r.act_gen[i]) for i, a in enumerate(ACTIONS)},
            "act_dist": {a: int(r.act_dist[i]) for i, a in enumerate(ACTIONS)},
            "seconds": float(r.seconds), "error": None, "complete": bool(r.complete),
            "narrow_levels": int(r.narrow_levels),
            "claim_mode": CLAIM_MODES.get(r.claim_mode, str(r.claim_mode)),
        }
        if self.cfg.seen_hbm_bytes:      # per-rank seen-set spill, summed over the ranks
            out.update(seen_flushes=int(r.seen_flushes), seen_cold_fps=int(r.seen_cold_fps),
                       seen_cold_runs=int(r.seen_cold_runs), seen_cold_queries=int(r.seen_cold_queries),
                       seen_cold_hits=int(r.seen_cold_hits))
        assert len(out["act_gen"]) == na
        if r.err_kind:
            tw = self.spec.tuple_words
            trace = []
            for i in range(r.trace_len):
                buf = (C.c_uint64 * tw)()
                check("kc_group_trace_tuple", self._lib.kc_group_trace_tuple(self._g, i, buf))
                trace.append([int(x) for x in buf])
            out.update(error={1: "assertion", 2: "invariant", 3: "deadlock"}[r.err_kind],
                       error_level=int(r.err_level), trace=trace, trace_len=int(r.trace_len))
            if r.err_kind == 1:
                out["error_action"] = ACTIONS[r.err_action]
            if r.err_kind == 2:
                out["error_invariant"] = INVARIANTS.get(r.err_invariant)
        return out

    def claim_times(self):
        """(k_claim ms, launches, parents) of this process's shards since the last call."""
        ms, n, p = C.c_double(), C.c_uint64(), C.c_uint64()
        tot = [0.0, 0, 0]
        for h in self._shards:
            check("kc_shard_claim_times", self._lib.kc_shard_claim_times(h, C.byref(ms), C.byref(n), C.byref(p)))
            tot = [tot[0] + ms.value, tot[1] + int(n.value), tot[2] + int(p.value)]
        return tuple(tot)

    def shard_result(self, i: int = 0) -> dict:
        r = KcResult()
        check("kc_shard_result", self._lib.kc_shard_result(self._shards[i], C.byref(r)))
        return {"generated": int(r.generated), "init": int(r.init), "distinct": int(r.distinct),
                "deferred": int(r.deferred_states)}

    def close(self) -> None:
        if self._g:
            self._lib.kc_group_destroy(self._g)
            self._g = C.c_void_p()
        for h in self._shards:
            self._lib.kc_shard_destroy(h)
        self._shards = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardedModelChecker:
    """Level-synchronous sharded BFS driver (collectives via torch.distributed)."""

    def __init__(self, cfg: ModelConfig, backend, group=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.cfg, self.be, self.group = cfg, backend, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if not 1 <= self.world <= MAX_WORLD:
            raise ValueError(f"sharded check: world size {self.world} outside 1..{MAX_WORLD}")
        self.dev = torch.device(backend.device_type, torch.cuda.current_device()) \
            if backend.device_type == "cuda" else torch.device("cpu")
        # exchange buffers in 8-byte words (records are whole words): element
        # counts stay 8x below byte counts (a uint8 all-to-all of > 1 GiB
        # came back corrupted through RCCL)
        self._send = torch.empty(0, dtype=torch.int64, device=self.dev)
        self._recv = torch.empty(0, dtype=torch.int64, device=self.dev)
        self.spec = Spec(cfg)
        if backend.device_type == "cuda" and hasattr(backend, "use_stream"):
            backend.use_stream(torch.cuda.current_stream())

    # -- collectives -----------------------------------------------------
    def _i64(self, vals: Sequence[int]):
        return self.torch.tensor(list(vals), dtype=self.torch.int64, device=self.dev)

    def _allreduce(self, vals: Sequence[int], op) -> List[int]:
        t = self._i64(vals)
        self.dist.all_reduce(t, op=op, group=self.group)
        return [int(x) for x in t.tolist()]

    def _buffer(self, name: str, nwords: int):
        buf = getattr(self, name)
        if buf.numel() < nwords:
            buf = self.torch.empty(max(nwords, 2 * buf.numel()), dtype=self.torch.int64, device=self.dev)
            setattr(self, name, buf)
        return buf

    # RCCL through torch returned only the first half of an all_to_all_single
    # larger than 1 GiB (MI355X, ROCm 7.2, torch 2.10): records move in
    # rounds of at most this many bytes per collective.
    A2A_ROUND_BYTES = 256 << 20

    def _gather_status(self, counts: List[int], n_new: int, err: int):
        """One all-gather per level: every rank's record counts per owner plus
        the (new states, error key) of the level it finished last.  Returns the
        counts matrix M[src][dst], the new-state counts and the error keys."""
        R = self.world
        if R == 1:
            return [list(counts)], [n_new], [err]
        cin = self._i64(list(counts) + [n_new, key_to_i64(err)])
        out = self.torch.empty(R * (R + 2), dtype=self.torch.int64, device=self.dev)
        self.dist.all_gather_into_tensor(out, cin, group=self.group)
        rows = out.view(R, R + 2).tolist()
        return [r[:R] for r in rows], [r[R] for r in rows], [i64_to_key(r[R + 1]) for r in rows]

    def _exchange(self, send, M: List[List[int]], rw: int):
        """All-to-all of the owner-grouped records given the counts matrix
        M[src][dst]; returns (recv, n_records), recv grouped by source rank."""
        torch, dist, R = self.torch, self.dist, self.world
        counts = M[self.rank]
        if R == 1:
            return send, counts[0]
        rcounts = [M[src][self.rank] for src in range(R)]
        recv = self._buffer("_recv", max(sum(rcounts), 1) * rw)
        q = max(1, self.A2A_ROUND_BYTES // (8 * rw * R))      # records per pair per round
        rounds = max(1, -(-max(max(r) for r in M) // q))
        if rounds == 1:
            dist.all_to_all_single(recv[: sum(rcounts) * rw], send[: sum(counts) * rw],
                                   output_split_sizes=[c * rw for c in rcounts],
                                   input_split_sizes=[c * rw for c in counts], group=self.group)
            return recv, sum(rcounts)
        sbase = [sum(counts[:d]) for d in range(R)]
        rbase = [sum(rcounts[:s]) for s in range(R)]
        for k in range(rounds):
            lo = k * q
            ins = [min(q, max(0, counts[d] - lo)) for d in range(R)]
            outs = [min(q, max(0, rcounts[s] - lo)) for s in range(R)]
            tin = torch.cat([send[(sbase[d] + lo) * rw: (sbase[d] + lo + ins[d]) * rw] for d in range(R)])
            tout = torch.empty(max(sum(outs), 1) * rw, dtype=torch.int64, device=self.dev)
            dist.all_to_all_single(tout[: sum(outs) * rw], tin,
                                   output_split_sizes=[c * rw for c in outs],
                                   input_split_sizes=[c * rw for c in ins], group=self.group)
            o = 0
            for s_ in range(R):
                if outs[s_]:
                    recv[(rbase[s_] + lo) * rw: (rbase[s_] + lo + outs[s_]) * rw].copy_(
                        tout[o * rw: (o + outs[s_]) * rw])
                o += outs[s_]
        return recv, sum(rcounts)

    def _sync(self):
        if self.dev.type == "cuda":
            self.torch.cuda.current_stream().synchronize()

    # -- the BFS ---------------------------------------------------------
    def run(self) -> dict:
        dist, be, rb = self.dist, self.be, self.be.record_bytes
        t0 = time.perf_counter()
        # One collective round trip per level: the all-gather that carries the
        # next level's record counts also carries the previous level's
        # (new states, error key).  Expanding a level before knowing that the
        # previous one ended the check is harmless (an empty frontier expands
        # to nothing; on an error the expansion is simply not used).
        # (After an error, the partial generated count therefore includes the
        # next level's expansion; TLC's partial counts at an error are not
        # deterministic either, and the error, its level and trace are.)
        prof = self._prof = {} if os.environ.get("KC_DRIVER_PROFILE") else None
        tick = time.perf_counter

        def lap(name, t):
            if prof is not None:
                prof[name] = prof.get(name, 0.0) + tick() - t
            return tick()

        # an Init violation is level 1's error, reported at level 1's gather
        # even when level 1 is not expanded (max_levels = 1)
        status_new = be.init()
        status_err = be.init_error()
        widths, level, err = [], 1, NONE_KEY
        self.records_sent = 0                             # to other ranks, this check
        rw = rb // 8                                      # record words
        while True:
            t = tick()
            last = bool(self.cfg.max_levels and level >= self.cfg.max_levels)
            if last:                                      # record the width, expand nothing
                counts, e1 = [0] * self.world, NONE_KEY
            else:
                counts, e1 = be.expand()                  # expand `level`
                if level == 1 and e1 != NONE_KEY and (e1 & 0xFF) == 0x12:
                    # an Init state violates an invariant: that is level 1's
                    # error (TLC checks Init before expanding anything), so it
                    # goes into this gather, ahead of any level-2 error
                    status_err, e1 = e1, NONE_KEY
            t = lap("expand", t)
            M, news, errs = self._gather_status(counts, status_new, status_err)
            t = lap("gather", t)
            err = min(errs)
            if err != NONE_KEY:                           # found while producing `level`
                level -= 1
                break
            total = sum(news)                             # width of `level`
            if total == 0:
                level -= 1
                break
            widths.append(total)
            if last:
                break
            self.records_sent += sum(counts) - counts[self.rank]
            send = self._buffer("_send", max(sum(counts), 1) * rw)
            be.pack(send)
            t = lap("pack", t)
            recv, nrecv = self._exchange(send, M, rw)
            if not getattr(be, "stream_ordered", False):
                self._sync()
            t = lap("exchange", t)
            n_new, e2 = be.insert(recv, nrecv)
            status_new, status_err = n_new, min(e1, e2)
            be.advance()
            t = lap("insert", t)
            level += 1
        seconds = time.perf_counter() - t0
        res = be.result()
        agg = self._allreduce(res["act_gen"] + res["act_dist"] +
                              [res["init"], res["generated"], res["distinct"]], dist.ReduceOp.SUM)
        na = len(ACTIONS)
        out = {
            "init": agg[2 * na], "generated": agg[2 * na] + agg[2 * na + 1],
            "distinct": agg[2 * na + 2], "depth": len(widths), "level_width": widths,
            "act_gen": dict(zip(ACTIONS, agg[:na])), "act_dist": dict(zip(ACTIONS, agg[na:2 * na])),
            "seconds": seconds, "error": None, "complete": err == NONE_KEY and not (
                self.cfg.max_levels and level >= self.cfg.max_levels),
        }
        if err != NONE_KEY:
            out.update(self._error(err, level))
        return out

    # -- counterexamples -------------------------------------------------
    def _query_parent(self, rank: int, level: int, idx: int) -> int:
        key = self.be.parent_key(level, idx) if self.rank == rank else 0
        t = self._i64([key - (1 << 64) if key >= (1 << 63) else key])
        self.dist.broadcast(t, src=rank, group=self.group)
        v = int(t.item())
        return v + (1 << 64) if v < 0 else v

    def _error(self, err: int, level: int) -> dict:
        kind = err & 0xff
        rank, pidx, pos = err >> 60, (err >> 16) & M44, (err >> 8) & 0xff
        if kind == 0x12:     # an Init state: its index in TLC's order is in the key
            s = self.spec.init()[pidx]
            return {"error_level": 1, "error": "invariant", "error_invariant": self.spec.check_invariants(s),
                    "trace": [[int(x) for x in s]], "trace_len": 1}
        path = []            # successor ordinals from an Init state
        r, idx, lvl = rank, pidx, level
        while lvl > 1:
            key = self._query_parent(r, lvl, idx)
            path.append((key >> 8) & 0xff)
            r, idx, lvl = key >> 60, (key >> 16) & M44, lvl - 1
        init_key = self._query_parent(r, 1, idx)
        states = [self.spec.init()[init_key & 0xffff]]
        for t in reversed(path):
            succ, _ = self.spec.successors(states[-1])
            states.append(succ[t][1])
        out = {"error_level": level}
        if kind == 2:                           # invariant violated by successor `pos`
            succ, _ = self.spec.successors(states[-1])
            states.append(succ[pos][1])
            out.update(error="invariant", error_invariant=self.spec.check_invariants(states[-1]),
                       error_level=level + 1)
        elif kind == 0x12:                      # an Init state violates an invariant
            out.update(error="invariant", error_invariant=self.spec.check_invariants(states[-1]),
                       error_level=1)
        elif kind == 1:
            _, fail = self.spec.successors(states[-1])
            out.update(error="assertion", error_action=fail)
        else:
            out.update(error="deadlock")
        out["trace"] = [[int(x) for x in s] for s in states]
        out["trace_len"] = len(states)
        return out


def pmc_ratio(workload: str):
    """PMC HBM bytes per algorithmic byte of the SHARDED k_claim, from the
    newest committed profiles/*_<workload>_sharded_rocprof_summary.json
    (tools/sharded_profile.py + tools/pmc_summary.py; bench.py cannot take
    PMC counters itself).  Streaming parent reads are counted at half by the
    counters (profiles/r02b_pmc_calibration.json) and restored here."""
    import glob
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    def run_order(f):      # r03z < r03aa < r03an: round, then tag length, then tag
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, os.path.basename(f))

    for f in reversed(sorted(glob.glob(os.path.join(root, "profiles", f"*_{workload}_sharded_rocprof_summary.json")),
                             key=run_order)):
        try:
            d = json.load(open(f))
            k, alg = d["kernels"]["k_claim"], d["algorithmic"]
            hbm = k["fetch_bytes_per_launch_raw"] + alg["stream_read_bytes_per_launch"] / 2 + \
                k["write_bytes_per_launch_raw"]
            return hbm / alg["algorithmic_bytes_per_launch"], os.path.relpath(f, root), d.get("build_id")
        except (OSError, ValueError, KeyError, ZeroDivisionError):
            continue
    return None, None, None


def claim_alg_bytes(parents: int, gen: int, deferred: int, records: int, S: int, record_bytes: int) -> int:
    """Algorithmic HBM bytes of the sharded k_claim, the
    engine's model (bench.py roofline_bfs) plus what only the sharded kernel
    writes: per expanded parent S (its state read); per generated successor
    64 (one probe line); on a deferred frontier per rebuilt parent S + 17 (its
    state written, its 8-B link and its parent's 8-B plan read, as the
    engine's 9-B trace entry + plan) and per parent 8 (its plan kept for the
    next level's rebuild); per remote representative the record it stages
    (record_bytes, written once by k_claim)."""
    b = parents * S + gen * 64 + records * record_bytes
    if deferred:
        b += deferred * (S + 17) + parents * 8
    return int(b)


def bench_sharded(args, kw: dict, desc: str, golden_check=None) -> Optional[dict]:
    """bench.py --gpus N: every rank checks its shard; rank 0 reports.  The
    counts are checked against the golden fixture (bench.golden_check); the
    roofline is k_claim's, per GPU (HIP events on every rank's k_claim
    launches, bytes as in bench.roofline_bfs); xGMI bytes are the records
    sent to other ranks."""
    import torch
    import torch.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rank, world = dist.get_rank(), dist.get_world_size()
    # the sharded loop's fast mode by default: the first
    # inserter of a state owns it (TLC -workers N semantics; counts, widths and
    # depth checked against the golden below); --deterministic-shards keeps the
    # (rank, parent)-ordered minimum claims and their settle passes
    first = not (getattr(args, "deterministic", False) or getattr(args, "deterministic_shards", False))
    cfg = ModelConfig(**kw, device=local, fpset_slots=1 << 20, timing=0 if args.no_timing else 2, first_claim=first)
    native = os.environ.get("KC_PY_DRIVER", "0") != "1"
    if native:                                        # the C++ level loop over RCCL
        mc = be = NativeShardedChecker(cfg, rank, world)
    else:                                             # the Python level loop (torch.distributed)
        be = HipShard(cfg, rank, world)
        mc = ShardedModelChecker(cfg, be)
    for _ in range(args.warmup):
        mc.run()
    be.claim_times()                                  # reset
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res, sent = None, 0
    for _ in range(args.steps):
        res = mc.run()
        sent += 0 if native else mc.records_sent
        if (not res["complete"] and not kw.get("max_levels")) or res["error"]:
            raise RuntimeError(f"sharded check incomplete: error={res['error']} depth={res['depth']}")
    torch.cuda.synchronize()
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    ms, launches, parents = be.claim_times()
    mine = be.shard_result() if native else be.result()
    S = 8 * Spec(cfg).state_words
    gen_local = mine["generated"] * args.steps        # successors of this rank's parents
    if native:
        sent = mc.records_sent * args.steps if rank == 0 else 0    # already summed over ranks
    # (records: rank 0 adds every rank's staged records, `sent` being global there)
    claim_bytes = claim_alg_bytes(parents, gen_local, mine.get("deferred", 0) * args.steps, sent, S, be.record_bytes)
    agg = torch.tensor([claim_bytes, int(ms * 1e6), launches, sent * be.record_bytes],
                       dtype=torch.int64, device="cuda")
    dist.all_reduce(agg, op=dist.ReduceOp.SUM)
    tot_bytes, tot_ns, tot_launch, xgmi = [int(x) for x in agg.tolist()]
    mc.close() if native else be.close()
    # the loop's per-level fixed cost, measured: Model_1 (124 levels, at most
    # 3,939 states wide) through the same loop and ranks is nearly all fixed
    # cost (launches, host syncs, collectives)
    fixed = None
    if native:
        m1 = NativeShardedChecker(ModelConfig(device=local, keep_trace=False), rank, world)
        try:
            m1.run()
            dist.barrier()
            t1 = time.perf_counter()
            for _ in range(3):
                r1 = m1.run()
            d1 = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device="cuda")
            dist.all_reduce(d1, op=dist.ReduceOp.MAX)
            fixed = {"model1_ms_per_check": round(float(d1.item()) / 3 * 1e3, 3), "levels": r1["depth"],
                     "us_per_level": round(float(d1.item()) / 3 / r1["depth"] * 1e6, 2),
                     "narrow_levels": r1.get("narrow_levels")}
        finally:
            m1.close()
    out = None
    if rank == 0:
        golden = golden_check(args.workload, res) if golden_check else None
        out = {
            "metric": "distinct states/sec (KubeAPI TLC BFS)",
            "value": round(res["distinct"] * args.steps / dt, 1),
            "unit": "distinct states/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3 / args.steps, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (the model's Init states; no external input)",
            "config": {"workload": desc, "model": f"nc={kw['nc']},np={kw['np']},ns={kw['ns']}"
                       + (f",max_levels={kw['max_levels']}" if kw.get("max_levels") else ""),
                       "distinct": res["distinct"], "generated": res["generated"],
                       "depth": res["depth"], "golden_check": golden,
                       "path": ("sharded, native C++ level loop over RCCL (kc_group_run)" if native else
                                "sharded, Python level loop over torch.distributed (kc_shard_* stages)"),
                       "parallelism": f"{world} GPUs, fingerprint-owner sharding, "
                                      "RCCL all-to-all per BFS level",
                       "xgmi_bytes_per_step": xgmi // max(args.steps, 1),
                       "xgmi_GBps_per_gpu": round(xgmi / max(args.steps, 1) / world
                                                  / (dt / args.steps) / 1e9, 2),
                       "per_level_fixed_cost": fixed,
                       "claims": ("first inserter (TLC -workers N semantics: same counts, widths and depth; "
                                  "the winning copy of a same-level duplicate is not deterministic)" if first else
                                  "(rank, parent, position) minimum (deterministic)"),
                       "claim_mode": res.get("claim_mode")},
        }
        if tot_ns > 0:
            achieved = tot_bytes / (tot_ns * 1e-9) / 1e9
            bpl = tot_bytes // max(tot_launch, 1)
            out["roofline"] = {"bound": "hbm", "achieved": round(achieved, 2), "peak": 8000.0,
                               "unit": "GB/s", "frac": round(achieved / 8000.0, 4), "traffic": None,
                               "kernel": "k_claim", "per": "GPU (all ranks' bytes / all ranks' k_claim time)",
                               "launches": tot_launch,
                               "avg_launch_us": round(tot_ns / 1e3 / max(tot_launch, 1), 2),
                               "bytes_per_launch": bpl}
            ratio, src, bid = pmc_ratio(args.workload)
            if ratio:
                from ._lib import build_id
                roof = out["roofline"]
                how = (f"{src}: PMC bytes / algorithmic bytes of the sharded k_claim = {ratio:.3f} "
                       "(rocprofv3 FETCH_SIZE + WRITE_SIZE passes over emulated ranks on one GPU), "
                       "times this run's algorithmic bytes per launch")
                if bid == build_id():
                    roof["traffic"] = int(ratio * bpl)
                    roof["traffic_unit"] = "HBM bytes per launch (PMC ratio of this build's kernel)"
                    roof["traffic_source"] = f"{how}; profile build {bid} = this build"
                else:                      # a profile of other kernels: not a measurement of these
                    roof["traffic_estimate"] = int(ratio * bpl)
                    roof["traffic_source"] = (f"{how}; profile build {bid or 'unrecorded'} is not this build "
                                              f"({build_id()}): an estimate only")
    dist.destroy_process_group()
    return out
