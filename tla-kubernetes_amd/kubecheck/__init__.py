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

from ._lib import (ACTIONS, ERR_KINDS, INVARIANTS, KcModelConfig, KcResult, KubecheckError,
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

    def to_c(self) -> KcModelConfig:
        c = KcModelConfig()
        for f in KcModelConfig._fields_:
            setattr(c, f[0], int(getattr(self, f[0])))
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
    trace: List[List[int]] = field(default_factory=list)
    trace_text: str = ""

    @property
    def distinct_per_sec(self) -> float:
        return self.distinct / self.seconds if self.seconds > 0 else 0.0


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
        outdeg_hist=[int(x) for x in r.outdeg_hist])


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
    """tlc2.tool.queue.StateQueue over fixed-width packed states in HBM."""

    def __init__(self, state_words: int, capacity: int, device: int = 0):
        self._lib = load()
        self.words = state_words
        self._h = C.c_void_p()
        check("kc_squeue_create", self._lib.kc_squeue_create(state_words, capacity, device, C.byref(self._h)))

    def enqueue(self, states: np.ndarray) -> None:
        a = np.ascontiguousarray(states, dtype=np.uint64).reshape(-1, self.words)
        check("kc_squeue_enqueue", self._lib.kc_squeue_enqueue(self._h, _u64(a), a.shape[0]))

    def dequeue(self, max_n: int) -> np.ndarray:
        out = np.zeros((max_n, self.words), dtype=np.uint64)
        n = C.c_size_t()
        check("kc_squeue_dequeue", self._lib.kc_squeue_dequeue(self._h, _u64(out), max_n, C.byref(n)))
        return out[: n.value]

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
