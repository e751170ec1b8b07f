"""ctypes wrapper of the CPU oracle (oracle/build/libkubeapi_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker.  The product never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libkubeapi_oracle.so")
NACT = 22
MAXLV = 4096
NBRANCH = 28
ACTIONS = [
    "DoRequest", "DoReply", "DoListRequest", "DoListReply", "CStart", "C1", "C10", "C11",
    "c12", "C13", "C2", "C3", "C8", "C6", "C7", "C4", "C5", "PVCStart", "PVCListedPVCs",
    "PVCHavePVCs", "PVCDone", "APIStart",
]
BRANCHES = [
    "CSTART_THEN", "CSTART_ELSE", "C1_START", "C1_C10", "C11_START", "C11_c12", "C13_START",
    "C13_C2", "C3_START", "C3_C8", "C8_C4", "C8_C6", "C7_START", "C7_C4", "PVCL_START",
    "PVCL_HAVE", "API_CREATE", "API_FORCE", "API_FORCE_REPLACE", "API_FORCE_CREATE", "API_GET",
    "API_GET_NOTFOUND", "API_DELETE", "API_UPDATE", "API_UPDATE_OK", "API_UPDATE_ERR",
    "API_LIST", "API_ASSERT",
]


class KoConfig(C.Structure):
    _fields_ = [("nc", C.c_int), ("np", C.c_int), ("ns", C.c_int), ("can_fail", C.c_int),
                ("can_timeout", C.c_int), ("check_deadlock", C.c_int), ("keep_trace", C.c_int),
                ("max_levels", C.c_int), ("max_distinct", C.c_uint64), ("variant", C.c_int),
                ("fp_bits", C.c_int), ("fpset_log2", C.c_int), ("progress", C.c_int),
                ("skip_inv", C.c_int), ("lost_update", C.c_int)]


class KoResult(C.Structure):
    _fields_ = [("init", C.c_uint64), ("generated", C.c_uint64), ("distinct", C.c_uint64),
                ("queue_left", C.c_uint64), ("depth", C.c_int), ("complete", C.c_int),
                ("act_gen", C.c_uint64 * NACT), ("act_dist", C.c_uint64 * NACT),
                ("cov_api", C.c_uint64), ("cov_req", C.c_uint64), ("cov_lreq", C.c_uint64),
                ("cov_objs", C.c_uint64), ("cov_api2", C.c_uint64),
                ("branch", C.c_uint64 * NBRANCH), ("outdeg_hist", C.c_uint64 * 32),
                ("newdeg_hist", C.c_uint64 * 32),
                ("nlevels", C.c_int), ("level_width", C.c_uint64 * MAXLV),
                ("err_kind", C.c_int), ("err_action", C.c_int), ("err_self", C.c_int),
                ("err_invariant", C.c_int), ("err_level", C.c_int), ("trace_len", C.c_int),
                ("seconds", C.c_double)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.ko_run.restype = C.c_void_p
        L.ko_run.argtypes = [C.POINTER(KoConfig), C.POINTER(KoResult)]
        L.ko_trace_text.restype = C.c_size_t
        L.ko_trace_text.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        L.ko_trace_tuple.restype = C.c_int
        L.ko_trace_tuple.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_uint64)]
        L.ko_free.argtypes = [C.c_void_p]
        L.ko_level_tuples.restype = C.c_uint64
        L.ko_level_tuples.argtypes = [C.POINTER(KoConfig), C.c_int, C.POINTER(C.c_uint64), C.c_uint64]
        L.ko_tuple_words.restype = C.c_int
        L.ko_tuple_words.argtypes = [C.POINTER(KoConfig)]
        L.ko_successors.restype = C.c_int
        L.ko_successors.argtypes = [C.POINTER(KoConfig), C.POINTER(C.c_uint64), C.POINTER(C.c_int),
                                    C.POINTER(C.c_uint64), C.c_int, C.POINTER(C.c_int)]
        L.ko_bench_sample.restype = C.c_double
        L.ko_bench_sample.argtypes = [C.POINTER(KoConfig), C.c_double, C.POINTER(C.c_uint64)]
        _lib = L
    return _lib


def config(nc=1, np_=1, ns=1, can_fail=True, can_timeout=True, check_deadlock=True,
           keep_trace=True, max_levels=0, variant=0, fp_bits=128, invariants=3) -> KoConfig:
    """invariants: bit 0 TypeOK, bit 1 OnlyOneVersion (the .cfg INVARIANT list),
    bit 2 the build-defined NoLostUpdate (with its lostUpdate history variable)."""
    return KoConfig(nc, np_, ns, int(can_fail), int(can_timeout), int(check_deadlock),
                    int(keep_trace), max_levels, 0, variant, fp_bits, 0, 0, 3 & ~invariants,
                    1 if invariants & 4 else 0)


def run(cfg: KoConfig) -> dict:
    r = KoResult()
    h = lib().ko_run(C.byref(cfg), C.byref(r))
    out = {
        "init": r.init, "generated": r.generated, "distinct": r.distinct,
        "queue_left": r.queue_left, "depth": r.depth, "complete": bool(r.complete),
        "act_gen": {a: int(r.act_gen[i]) for i, a in enumerate(ACTIONS)},
        "act_dist": {a: int(r.act_dist[i]) for i, a in enumerate(ACTIONS)},
        "cov": {"api": r.cov_api, "req": r.cov_req, "lreq": r.cov_lreq, "objs": r.cov_objs,
                "api2": r.cov_api2},
        "branch": {b: int(r.branch[i]) for i, b in enumerate(BRANCHES)},
        "level_width": [int(r.level_width[i]) for i in range(r.nlevels)],
        "newdeg_hist": [int(x) for x in r.newdeg_hist],
        "err_kind": r.err_kind, "err_action": ACTIONS[r.err_action] if r.err_action >= 0 else None,
        "err_self": r.err_self, "err_invariant": r.err_invariant, "err_level": r.err_level,
        "trace_len": r.trace_len, "seconds": r.seconds, "trace": [], "trace_text": "",
    }
    if h:
        w = lib().ko_tuple_words(C.byref(cfg))
        for i in range(r.trace_len):
            t = (C.c_uint64 * w)()
            lib().ko_trace_tuple(h, i, t)
            out["trace"].append(list(t))
        n = lib().ko_trace_text(h, None, 0)
        buf = C.create_string_buffer(n + 1)
        lib().ko_trace_text(h, buf, n + 1)
        out["trace_text"] = buf.value.decode()
        lib().ko_free(h)
    return out


def level_tuples(cfg: KoConfig, level: int) -> np.ndarray:
    L = lib()
    n = L.ko_level_tuples(C.byref(cfg), level, None, 0)
    w = L.ko_tuple_words(C.byref(cfg))
    out = np.zeros((n, w), dtype=np.uint64)
    L.ko_level_tuples(C.byref(cfg), level, out.ctypes.data_as(C.POINTER(C.c_uint64)), n)
    return out


def successors(cfg: KoConfig, tup):
    L = lib()
    w = L.ko_tuple_words(C.byref(cfg))
    t = np.ascontiguousarray(tup, dtype=np.uint64)
    acts = (C.c_int * 64)()
    out = np.zeros((64, w), dtype=np.uint64)
    fail = C.c_int(-1)
    n = L.ko_successors(C.byref(cfg), t.ctypes.data_as(C.POINTER(C.c_uint64)), acts,
                        out.ctypes.data_as(C.POINTER(C.c_uint64)), 64, C.byref(fail))
    if n < 0:
        return None, ACTIONS[fail.value]
    return [(ACTIONS[acts[i]], out[i]) for i in range(n)], None


class KoParResult(C.Structure):
    _fields_ = [("distinct", C.c_uint64), ("generated", C.c_uint64), ("levels", C.c_int),
                ("complete", C.c_int), ("set_full", C.c_int), ("threads", C.c_int),
                ("seconds", C.c_double), ("fp_bits", C.c_int), ("depth", C.c_int),
                ("level_width", C.c_uint64 * 4096)]


def bench_parallel(cfg: KoConfig, threads: int, seconds: float) -> dict:
    """Multi-core comparator (ko_bench_parallel): BFS from Init on `threads`
    host threads for about `seconds`."""
    L = lib()
    L.ko_bench_parallel.restype = C.c_double
    L.ko_bench_parallel.argtypes = [C.POINTER(KoConfig), C.c_int, C.c_double, C.POINTER(KoParResult)]
    r = KoParResult()
    rate = L.ko_bench_parallel(C.byref(cfg), threads, seconds, C.byref(r))
    return {"rate": rate, "distinct": r.distinct, "generated": r.generated, "levels": r.levels,
            "complete": bool(r.complete), "set_full": bool(r.set_full), "threads": r.threads,
            "seconds": r.seconds}


def bench_sample(cfg: KoConfig, seconds: float):
    done = C.c_uint64()
    rate = lib().ko_bench_sample(C.byref(cfg), seconds, C.byref(done))
    return rate, done.value


class KoFpsetCpuResult(C.Structure):
    _fields_ = [("slots", C.c_uint64), ("inserted", C.c_uint64), ("duplicates", C.c_uint64),
                ("found", C.c_uint64), ("threads", C.c_int), ("insert_seconds", C.c_double),
                ("lookup_seconds", C.c_double), ("inserts_per_s", C.c_double), ("lookups_per_s", C.c_double)]


def fpset_stress_cpu(n: int, load: float, threads: int, seed: int = 0x5EED0000) -> dict:
    """Host FPSet comparator (fpset_cpu.c): n distinct fingerprints inserted by
    `threads` threads into one table at `load`, then n lookups (half present)."""
    L = lib()
    L.ko_fpset_stress_cpu.restype = C.c_int
    L.ko_fpset_stress_cpu.argtypes = [C.c_uint64, C.c_double, C.c_int, C.c_uint64, C.POINTER(KoFpsetCpuResult)]
    r = KoFpsetCpuResult()
    rc = L.ko_fpset_stress_cpu(n, load, threads, seed, C.byref(r))
    if rc != 0:
        raise RuntimeError(f"ko_fpset_stress_cpu failed ({rc})")
    return {f[0]: getattr(r, f[0]) for f in KoFpsetCpuResult._fields_}
