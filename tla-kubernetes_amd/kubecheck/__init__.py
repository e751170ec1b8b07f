"""kubecheck — MI355X-native BFS model checker for KubeAPI.tla.

Host-side mirror of the reference's checking surface (TLC 2.16 as run on
KubeAPI.toolbox/Model_1, MC.out:2-5):

* :class:`FPSet`        — tlc2.tool.fp.FPSet (put / contains / size / checkFPs),
                          backed by the HBM open-addressing set.
* :class:`StateQueue`   — tlc2.tool.queue.StateQueue over packed states in HBM.
* :class:`ModelChecker` — tlc2.TLC's BFS safety check of Spec with the Model_1
                          inputs (MC.cfg / MC.tla), reporting the same counts
                          (MC.out:1098), depth (:1101), per-action coverage
                          (:78-621) and counterexample traces.
* :mod:`kubecheck.tlc`  — TLC-style command line (``-config MC.cfg MC``) with
                          ``-tool`` message output.

All compute runs in libkubecheck.so (HIP, gfx950).  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from ._lib import (ACTIONS, ERR_KINDS, INVARIANTS, KcModelConfig, KcResult, KcSqueueConfig,
                   KcSqueueStats, KubecheckError,
                   check, load)

__all__ = ["ModelConfig", "ModelChecker", "CheckResult", "FPSet", "StateQueue", "Spec",
           "KubecheckError", "ACTIONS", "load", "device_count", "stress_fps_dev", "stress_fp"]


def device_count() -> int:
    return load().kc_device_count()


@dataclass
class ModelConfig:
    """A KubeAPI model: Model_1 is nc=np=ns=1 with both constants TRUE."""
    nc: int = 1                 # clients            (KubeAPI.tla:161)
    np: int = 1                 # PVC controllers    (KubeAPI.tla:225)
    ns: int = 1                 # API servers        (KubeAPI.tla:268)
    can_fail: bool = True       # REQUESTS_CAN_FAIL    (MC.tla:5-7)
    can_timeout: bool = True    # REQUESTS_CAN_TIMEOUT (MC.tla:10-12)
    check_deadlock: bool = True # KubeAPI___Model_1.launch:16
    variant: int = 0            # seeded bugs 1-5 (include/kubecheck.h); 0 = KubeAPI.tla as written
    device: int = 0
    keep_trace: bool = True
    max_levels: int = 0
    fpset_slots: int = 0
    chunk_states: int = 0
    verbose: int = 0
    timing: int = 0             # HIP-event timing (kernel_times()): 1 every kernel, 2 k_claim only
    invariants: int = 3         # MC.cfg INVARIANT: bit 0 TypeOK, bit 1 OnlyOneVersion (0 = none)
    # frontier spill (TLC's DiskStateQueue role): > 0 keeps the frontiers in a
    # StateQueue with this HBM budget; past it segments go to pinned host RAM
    # (frontier_host_bytes, 0 = unlimited), then to files in spill_dir
    frontier_hbm_bytes: int = 0
    frontier_host_bytes: int = 0
    frontier_segment_states: int = 0   # parents per chunk / states per segment (0 = 2^22)
    spill_dir: Optional[str] = None
    trace_host: bool = False    # the trace file (9 B per state) in pinned host RAM
    # seen-set spill (TLC's OffHeapDiskFPSet role): > 0 caps the seen-set's HBM;
    # older fingerprints go to sorted runs in pinned host RAM (seen_host_bytes,
    # 0 = unlimited), then to files in spill_dir
    seen_hbm_bytes: int = 0
    seen_host_bytes: int = 0
    # sharded runs at R > 1: claims in sequential-BFS order, so errors and
    # traces equal TLC -workers 1's (a per-level all-reduce and sort)
    tlc_order: bool = False
    # the first inserter of a state owns it (TLC -workers N semantics: same
    # counts and trace lengths, no settle passes; the winning copy of a
    # same-level duplicate is not deterministic).  The engine's in-HBM wide
    # levels and every counted level of the sharded loop (not with tlc_order
    # or the seen-set spill there); CheckResult.claim_mode says what ran
    first_claim: bool = False

    def to_c(self) -> KcModelConfig:
        c = KcModelConfig()
        for f in KcModelConfig._fields_:
            if f[0] == "spill_dir":
                continue
            setattr(c, f[0], int(getattr(self, f[0])))
        # the C string must outlive the engine's use of the config (copied at create)
        c.spill_dir = self.spill_dir.encode() if self.spill_dir else None
        return c

    @property
    def name(self) -> str:
        return f"KubeAPI(nc={self.nc},np={self.np},ns={self.ns})"


@dataclass
class CheckResult:
    init: int
    generated: int
    distinct: int
    queue_left: int
    depth: int
    complete: bool
    act_gen: Dict[str, int]
    act_dist: Dict[str, int]
    level_width: List[int]
    error: Optional[str]              # None, "assertion", "invariant", "deadlock"
    error_action: Optional[str]
    error_self: int
    error_invariant: Optional[str]
    error_level: int
    trace_len: int
    seconds: float
    collision_optimistic: float
    fpset_slots: int
    peak_frontier: int
    fpset_probes: int = 0
    batch_inserts: int = 0
    levels_chunks: int = 0
    outdeg_hist: List[int] = field(default_factory=list)
    frontier_spilled_bytes: int = 0
    frontier_reloaded_bytes: int = 0
    frontier_peak_hbm_bytes: int = 0
    seen: Dict[str, float] = field(default_factory=dict)   # seen-set spill statistics (seen_* fields)
    cand_overflow_records: int = 0
    cand_buffer_peak_bytes: int = 0
    deferred_states: int = 0       # frontier states rebuilt inside k_claim (deferred frontier)
    defer_fallback: bool = False   # the run was redone on the materialising path
    defer_redo_level: int = 0      # ... starting from this level (1 = Init; 0 = no redo)
    narrow_levels: int = 0         # levels run by the device-driven narrow kernel
    claim_mode: str = "minimum"    # the claims that ran: "minimum" (sequential-BFS / rank-major), "first", "tlc"
    trace: List[List[int]] = field(default_factory=list)
    trace_text: str = ""

    @property
    def distinct_per_sec(self) -> float:
        return self.distinct / self.seconds if self.seconds > 0 else 0.0


CLAIM_MODES = {0: "minimum", 1: "first", 2: "tlc"}


def _result(r: KcResult) -> CheckResult:
    return CheckResult(
        init=r.init, generated=r.generated, distinct=r.distinct, queue_left=r.queue_left,
        depth=r.depth, complete=bool(r.complete),
        act_gen={a: int(r.act_gen[i]) for i, a in enumerate(ACTIONS)},
        act_dist={a: int(r.act_dist[i]) for i, a in enumerate(ACTIONS)},
        level_width=[int(r.level_width[i]) for i in range(r.nlevels)],
        error=ERR_KINDS.get(r.err_kind),
        error_action=ACTIONS[r.err_action] if 0 <= r.err_action < len(ACTIONS) else None,
        error_self=r.err_self,
        error_invariant=INVARIANTS.get(r.err_invariant),
        error_level=r.err_level, trace_len=r.trace_len, seconds=r.seconds,
        collision_optimistic=r.collision_optimistic, fpset_slots=r.fpset_slots,
        peak_frontier=r.peak_frontier, fpset_probes=r.fpset_probes,
        batch_inserts=r.batch_inserts, levels_chunks=r.levels_chunks,
        outdeg_hist=[int(x) for x in r.outdeg_hist],
        frontier_spilled_bytes=r.frontier_spilled_bytes, frontier_reloaded_bytes=r.frontier_reloaded_bytes,
        frontier_peak_hbm_bytes=r.frontier_peak_hbm_bytes,
        seen={f[0][5:]: getattr(r, f[0]) for f in KcResult._fields_ if f[0].startswith("seen_")},
        cand_overflow_records=r.cand_overflow_records, cand_buffer_peak_bytes=r.cand_buffer_peak_bytes,
        deferred_states=r.deferred_states, defer_fallback=bool(r.defer_fallback),
        defer_redo_level=int(r.defer_redo_level), narrow_levels=int(r.narrow_levels),
        claim_mode=CLAIM_MODES.get(r.claim_mode, str(r.claim_mode)))


class ModelChecker:
    """BFS safety checker (TLC's ModelChecker for this spec) on one GPU."""

    def __init__(self, cfg: Optional[ModelConfig] = None, **kw):
        self.cfg = cfg or ModelConfig(**kw)
        self._lib = load()
        self._h = C.c_void_p()
        self._c = self.cfg.to_c()
        check("kc_engine_create", self._lib.kc_engine_create(C.byref(self._c), C.byref(self._h)))
        self.tuple_words = self._lib.kc_spec_tuple_words(self.cfg.nc, self.cfg.np, self.cfg.ns)

    def capture_level(self, level: int) -> None:
        check("kc_engine_capture_level", self._lib.kc_engine_capture_level(self._h, level))

    def run(self) -> CheckResult:
        r = KcResult()
        check("kc_engine_run", self._lib.kc_engine_run(self._h, C.byref(r)))
        res = _result(r)
        if res.error is not None and res.trace_len:
            res.trace = [self.trace_tuple(i) for i in range(res.trace_len)]
            n = self._lib.kc_engine_trace_text(self._h, None, 0)
            buf = C.create_string_buffer(n)
            self._lib.kc_engine_trace_text(self._h, buf, n)
            res.trace_text = buf.value.decode()
        return res

    def trace_tuple(self, i: int) -> List[int]:
        out = (C.c_uint64 * self.tuple_words)()
        check("kc_engine_trace_tuple", self._lib.kc_engine_trace_tuple(self._h, i, out))
        return list(out)

    def level_tuples(self, level: int) -> np.ndarray:
        n = check("kc_engine_level_tuples", self._lib.kc_engine_level_tuples(self._h, level, None, 0))
        out = np.zeros((n, self.tuple_words), dtype=np.uint64)
        check("kc_engine_level_tuples", self._lib.kc_engine_level_tuples(
            self._h, level, out.ctypes.data_as(C.POINTER(C.c_uint64)), n))
        return out

    def kernel_times(self):
        ms = (C.c_double * 4)()
        cnt = (C.c_uint64 * 4)()
        check("kc_engine_kernel_times", self._lib.kc_engine_kernel_times(self._h, ms, cnt))
        names = ["expand", "resolve", "scan", "emit"]
        return {k: (ms[i], int(cnt[i])) for i, k in enumerate(names)}

    def check_fps(self):
        """TLC checkFPs on the last run's seen-set: (min gap, 1/min gap)."""
        gap, prob = C.c_uint64(), C.c_double()
        check("kc_engine_check_fps", self._lib.kc_engine_check_fps(self._h, C.byref(gap), C.byref(prob)))
        return int(gap.value), prob.value

    def narrow_times(self):
        """(ms, launches, levels) of the narrow-level kernel in the last run."""
        ms, n, lv = C.c_double(), C.c_uint64(), C.c_uint64()
        check("kc_engine_narrow_times", self._lib.kc_engine_narrow_times(self._h, C.byref(ms), C.byref(n),
                                                                          C.byref(lv)))
        return ms.value, int(n.value), int(lv.value)

    def close(self) -> None:
        if self._h:
            self._lib.kc_engine_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _stream(stream):
    return C.c_void_p(stream.cuda_stream if stream is not None else 0)


def stress_fps_dev(seed: int, kind: int, n_ins: int, start: int, n: int, out, stream=None) -> None:
    """Stress stream entries [start, start+n) into a device tensor
    (kind 0 = inserts, 1 = lookups; kc_stress_fps_dev)."""
    check("kc_stress_fps_dev", load().kc_stress_fps_dev(seed, kind, n_ins, start, n,
                                                         C.c_void_p(out.data_ptr()), _stream(stream)))


def stress_fp(seed: int, kind: int, n_ins: int, i: int) -> int:
    return int(load().kc_stress_fp(seed, kind, n_ins, i))


def _u64(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


class FPSet:
    """tlc2.tool.fp.FPSet on HBM.  put() returns True iff fp was already present."""

    def __init__(self, capacity: int = 1 << 20, device: int = 0):
        self._lib = load()
        self._h = C.c_void_p()
        check("kc_fpset_create", self._lib.kc_fpset_create(int(capacity), device, C.byref(self._h)))

    def put_batch(self, fps) -> np.ndarray:
        a = np.ascontiguousarray(fps, dtype=np.uint64)
        seen = np.zeros(a.shape[0], dtype=np.uint8)
        check("kc_fpset_put_batch", self._lib.kc_fpset_put_batch(
            self._h, _u64(a), a.shape[0], seen.ctypes.data_as(C.POINTER(C.c_uint8))))
        return seen.astype(bool)

    def contains_batch(self, fps) -> np.ndarray:
        a = np.ascontiguousarray(fps, dtype=np.uint64)
        seen = np.zeros(a.shape[0], dtype=np.uint8)
        check("kc_fpset_contains_batch", self._lib.kc_fpset_contains_batch(
            self._h, _u64(a), a.shape[0], seen.ctypes.data_as(C.POINTER(C.c_uint8))))
        return seen.astype(bool)

    def put(self, fp: int) -> bool:
        """TLC FPSet.put(long): thread-safe; concurrent callers are
        flat-combined into one batch launch (kc_fpset_put)."""
        seen = C.c_int()
        check("kc_fpset_put", self._lib.kc_fpset_put(self._h, int(fp) & (2**64 - 1), C.byref(seen)))
        return bool(seen.value)

    def contains(self, fp: int) -> bool:
        seen = C.c_int()
        check("kc_fpset_contains", self._lib.kc_fpset_contains(self._h, int(fp) & (2**64 - 1), C.byref(seen)))
        return bool(seen.value)

    def combine_rounds(self) -> int:
        """Batches launched so far by put()/contains()."""
        return int(self._lib.kc_fpset_combine_rounds(self._h))

    # -- device-resident batches (torch tensors of int64 on this set's GPU)
    def insert_count_dev(self, fps, n: int, stream=None) -> int:
        """Insert the first n fps of a device tensor; returns how many were new."""
        out = C.c_uint64()
        check("kc_fpset_insert_count_dev", self._lib.kc_fpset_insert_count_dev(
            self._h, C.c_void_p(fps.data_ptr()), n, C.byref(out), _stream(stream)))
        return int(out.value)

    def contains_count_dev(self, fps, n: int, stream=None) -> int:
        out = C.c_uint64()
        check("kc_fpset_contains_count_dev", self._lib.kc_fpset_contains_count_dev(
            self._h, C.c_void_p(fps.data_ptr()), n, C.byref(out), _stream(stream)))
        return int(out.value)

    def partition_dev(self, fps, n: int, world: int, out, stream=None) -> List[int]:
        """Stable counting sort of n device fps by owner rank into `out`;
        returns the per-owner counts."""
        counts = (C.c_uint64 * world)()
        check("kc_fpset_partition_dev", self._lib.kc_fpset_partition_dev(
            self._h, C.c_void_p(fps.data_ptr()), n, world, C.c_void_p(out.data_ptr()), counts,
            _stream(stream)))
        return [int(x) for x in counts]

    def size(self) -> int:
        return int(self._lib.kc_fpset_size(self._h))

    def capacity(self) -> int:
        return int(self._lib.kc_fpset_capacity(self._h))

    def checkFPs(self) -> float:
        gap = C.c_uint64()
        prob = C.c_double()
        check("kc_fpset_check_fps", self._lib.kc_fpset_check_fps(self._h, C.byref(gap), C.byref(prob)))
        self.min_gap = gap.value
        return prob.value

    def stress(self, seed: int, n: int, batch: int, n_lookup: int):
        ti, tl, found = C.c_double(), C.c_double(), C.c_uint64()
        check("kc_fpset_stress", self._lib.kc_fpset_stress(
            self._h, seed, n, batch, n_lookup, C.byref(ti), C.byref(tl), C.byref(found)))
        return ti.value, tl.value, found.value

    def close(self) -> None:
        if self._h:
            self._lib.kc_fpset_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class StateQueue:
    """tlc2.tool.queue.StateQueue (the recorded run's DiskStateQueue,
    MC.out:5): a FIFO of fixed-width packed states in segments over HBM,
    pinned host RAM past `hbm_bytes`, and spill files in `spill_dir` past
    `host_bytes` (include/kubecheck.h kc_squeue_*).  Host-array calls are
    synchronous; the ``*_dev`` calls take device pointers or CUDA tensors and
    an optional HIP stream (None = the queue's own stream, ordered with the
    default stream)."""

    def __init__(self, state_words: int, capacity: int = 0, device: int = 0, *, segment_states: int = 0,
                 hbm_bytes: int = 0, host_bytes: int = 0, spill_dir: Optional[str] = None):
        self._lib = load()
        self.words = state_words
        self._h = C.c_void_p()
        if capacity and not (segment_states or hbm_bytes or host_bytes or spill_dir):
            check("kc_squeue_create", self._lib.kc_squeue_create(state_words, capacity, device, C.byref(self._h)))
            return
        c = KcSqueueConfig(state_words=state_words, device=device, segment_states=segment_states or capacity,
                           hbm_bytes=hbm_bytes, host_bytes=host_bytes,
                           spill_dir=spill_dir.encode() if spill_dir else None)
        check("kc_squeue_create2", self._lib.kc_squeue_create2(C.byref(c), C.byref(self._h)))

    @staticmethod
    def _ptr(x) -> int:
        return int(x.data_ptr()) if hasattr(x, "data_ptr") else int(x)

    @staticmethod
    def _st(stream):
        if stream is None:
            return None
        return C.c_void_p(int(getattr(stream, "cuda_stream", stream)))

    def enqueue(self, states: np.ndarray) -> None:
        a = np.ascontiguousarray(states, dtype=np.uint64).reshape(-1, self.words)
        check("kc_squeue_enqueue", self._lib.kc_squeue_enqueue(self._h, _u64(a), a.shape[0]))

    def dequeue(self, max_n: int) -> np.ndarray:
        out = np.zeros((max_n, self.words), dtype=np.uint64)
        n = C.c_size_t()
        check("kc_squeue_dequeue", self._lib.kc_squeue_dequeue(self._h, _u64(out), max_n, C.byref(n)))
        return out[: n.value]

    def enqueue_dev(self, states, n: Optional[int] = None, stream=None) -> None:
        """Append n states from device memory (a CUDA tensor of n x words
        64-bit values, or a device pointer with n given)."""
        if n is None:
            n = states.numel() // self.words
        check("kc_squeue_enqueue_dev",
              self._lib.kc_squeue_enqueue_dev(self._h, C.c_void_p(self._ptr(states)), n, self._st(stream)))

    def dequeue_dev(self, out, max_n: int, stream=None) -> int:
        """Move up to max_n head states into device memory; returns the count."""
        got = C.c_size_t()
        check("kc_squeue_dequeue_dev", self._lib.kc_squeue_dequeue_dev(
            self._h, C.c_void_p(self._ptr(out)), max_n, C.byref(got), self._st(stream)))
        return got.value

    def reserve_dev(self, n: int, stream=None) -> int:
        """Device pointer to n writable states at the tail (then commit)."""
        p = C.c_void_p()
        check("kc_squeue_reserve_dev", self._lib.kc_squeue_reserve_dev(self._h, n, C.byref(p), self._st(stream)))
        return int(p.value)

    def commit(self, n: int, stream=None) -> None:
        check("kc_squeue_commit", self._lib.kc_squeue_commit(self._h, n, self._st(stream)))

    def front_dev(self, offset: int, max_n: int, stream=None):
        """(device pointer, count) of a contiguous run `offset` states after
        the head; count may be < max_n at a segment end."""
        p = C.c_void_p()
        got = C.c_size_t()
        check("kc_squeue_front_dev", self._lib.kc_squeue_front_dev(
            self._h, offset, max_n, C.byref(p), C.byref(got), self._st(stream)))
        return int(p.value or 0), got.value

    def pop(self, n: int, stream=None) -> None:
        check("kc_squeue_pop", self._lib.kc_squeue_pop(self._h, n, self._st(stream)))

    def peek(self, offset: int, n: int) -> np.ndarray:
        out = np.zeros((n, self.words), dtype=np.uint64)
        check("kc_squeue_peek", self._lib.kc_squeue_peek(self._h, offset, n, _u64(out), None))
        return out

    def stats(self) -> Dict[str, int]:
        st = KcSqueueStats()
        check("kc_squeue_get_stats", self._lib.kc_squeue_get_stats(self._h, C.byref(st)))
        return {f[0]: int(getattr(st, f[0])) for f in KcSqueueStats._fields_}

    def size(self) -> int:
        return int(self._lib.kc_squeue_size(self._h))

    def close(self) -> None:
        if self._h:
            self._lib.kc_squeue_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Spec:
    """Host access to the lowered spec (canonical tuples; no GPU needed)."""

    def __init__(self, cfg: Optional[ModelConfig] = None, **kw):
        self.cfg = cfg or ModelConfig(**kw)
        self._lib = load()
        self._c = self.cfg.to_c()
        self.tuple_words = check("kc_spec_tuple_words",
                                 self._lib.kc_spec_tuple_words(self.cfg.nc, self.cfg.np, self.cfg.ns))
        self.state_words = check("kc_spec_state_words",
                                 self._lib.kc_spec_state_words(self.cfg.nc, self.cfg.np, self.cfg.ns))

    def init(self) -> np.ndarray:
        n = check("kc_spec_init", self._lib.kc_spec_init(C.byref(self._c), None, 0))
        out = np.zeros((n, self.tuple_words), dtype=np.uint64)
        self._lib.kc_spec_init(C.byref(self._c), _u64(out), n)
        return out

    def successors(self, tup):
        t = np.ascontiguousarray(tup, dtype=np.uint64)
        cap = 64
        acts = (C.c_int * cap)()
        out = np.zeros((cap, self.tuple_words), dtype=np.uint64)
        fail = C.c_int(-1)
        n = self._lib.kc_spec_successors(C.byref(self._c), _u64(t), acts, _u64(out), cap, C.byref(fail))
        if n == -2:
            return None, ACTIONS[fail.value]
        check("kc_spec_successors", n)
        return [(ACTIONS[acts[i]], out[i]) for i in range(n)], None

    def check_invariants(self, tup) -> Optional[str]:
        t = np.ascontiguousarray(tup, dtype=np.uint64)
        r = self._lib.kc_spec_check(C.byref(self._c), _u64(t))
        if r < -1:
            check("kc_spec_check", r)
        return INVARIANTS.get(r)

    def fingerprint(self, tup) -> int:
        t = np.ascontiguousarray(tup, dtype=np.uint64)
        fp = C.c_uint64()
        check("kc_spec_fingerprint", self._lib.kc_spec_fingerprint(C.byref(self._c), _u64(t), C.byref(fp)))
        return fp.value

    def fp_selfcheck(self, tup) -> int:
        """Successors whose incremental (kernel) fingerprint differs from the
        full one; 0 expected."""
        t = np.ascontiguousarray(tup, dtype=np.uint64)
        return check("kc_spec_fp_selfcheck", self._lib.kc_spec_fp_selfcheck(C.byref(self._c), _u64(t)))

    def pack(self, tup) -> np.ndarray:
        t = np.ascontiguousarray(tup, dtype=np.uint64)
        out = np.zeros(self.state_words, dtype=np.uint64)
        check("kc_spec_pack", self._lib.kc_spec_pack(C.byref(self._c), _u64(t), _u64(out)))
        return out

    def unpack(self, packed) -> np.ndarray:
        p = np.ascontiguousarray(packed, dtype=np.uint64)
        out = np.zeros(self.tuple_words, dtype=np.uint64)
        check("kc_spec_unpack", self._lib.kc_spec_unpack(C.byref(self._c), _u64(p), _u64(out)))
        return out
