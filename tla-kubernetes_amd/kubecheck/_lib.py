"""ctypes binding of libkubecheck.so (include/kubecheck.h).

The library is built in-tree (tla-kubernetes_amd/csrc/Makefile ->
tla-kubernetes_amd/kubecheck/lib/libkubecheck.so).  There is no Python or CPU
fallback for the model checker: if the library is missing, importing the
product raises, and engine calls on a machine without a GPU fail with ENODEV.
"""
from __future__ import annotations

import ctypes as C
import os

LIB_PATH = os.environ.get("KUBECHECK_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "lib", "libkubecheck.so")

KC_NACTIONS = 22
KC_MAX_LEVELS = 4096

ACTIONS = [
    "DoRequest", "DoReply", "DoListRequest", "DoListReply", "CStart", "C1", "C10", "C11",
    "c12", "C13", "C2", "C3", "C8", "C6", "C7", "C4", "C5", "PVCStart", "PVCListedPVCs",
    "PVCHavePVCs", "PVCDone", "APIStart",
]

ERR_KINDS = {0: None, 1: "assertion", 2: "invariant", 3: "deadlock"}
INVARIANTS = {0: "TypeOK", 1: "OnlyOneVersion", 2: "NoLostUpdate"}


class KcModelConfig(C.Structure):
    _fields_ = [
        ("nc", C.c_int), ("np", C.c_int), ("ns", C.c_int),
        ("can_fail", C.c_int), ("can_timeout", C.c_int), ("check_deadlock", C.c_int),
        ("variant", C.c_int), ("device", C.c_int), ("keep_trace", C.c_int),
        ("max_levels", C.c_int), ("fpset_slots", C.c_uint64), ("chunk_states", C.c_uint64),
        ("verbose", C.c_int), ("timing", C.c_int), ("invariants", C.c_int),
        ("frontier_hbm_bytes", C.c_uint64), ("frontier_host_bytes", C.c_uint64),
        ("frontier_segment_states", C.c_uint64), ("spill_dir", C.c_char_p), ("trace_host", C.c_int),
        ("seen_hbm_bytes", C.c_uint64), ("seen_host_bytes", C.c_uint64),
        ("tlc_order", C.c_int),
        ("first_claim", C.c_int),
    ]


class KcResult(C.Structure):
    _fields_ = [
        ("init", C.c_uint64), ("generated", C.c_uint64), ("distinct", C.c_uint64),
        ("queue_left", C.c_uint64), ("depth", C.c_int), ("complete", C.c_int),
        ("act_gen", C.c_uint64 * KC_NACTIONS), ("act_dist", C.c_uint64 * KC_NACTIONS),
        ("nlevels", C.c_int), ("level_width", C.c_uint64 * KC_MAX_LEVELS),
        ("err_kind", C.c_int), ("err_action", C.c_int), ("err_self", C.c_int),
        ("err_invariant", C.c_int), ("err_level", C.c_int), ("trace_len", C.c_int),
        ("seconds", C.c_double), ("collision_optimistic", C.c_double),
        ("fpset_slots", C.c_uint64), ("peak_frontier", C.c_uint64),
        ("fpset_probes", C.c_uint64), ("batch_inserts", C.c_uint64),
        ("levels_chunks", C.c_uint64), ("outdeg_hist", C.c_uint64 * 16),
        ("frontier_spilled_bytes", C.c_uint64), ("frontier_reloaded_bytes", C.c_uint64),
        ("frontier_peak_hbm_bytes", C.c_uint64),
        ("seen_flushes", C.c_uint64), ("seen_cold_fps", C.c_uint64), ("seen_cold_runs", C.c_uint64),
        ("seen_cold_queries", C.c_uint64), ("seen_cold_hits", C.c_uint64), ("seen_merges", C.c_uint64),
        ("seen_filter_tests", C.c_uint64), ("seen_filter_passed", C.c_uint64),
        ("seen_disk_bytes", C.c_uint64), ("seen_peak_hbm_bytes", C.c_uint64), ("seen_seconds", C.c_double),
        ("seen_flush_seconds", C.c_double), ("seen_merge_seconds", C.c_double), ("seen_check_seconds", C.c_double),
        ("cand_overflow_records", C.c_uint64), ("cand_buffer_peak_bytes", C.c_uint64),
        ("deferred_states", C.c_uint64), ("defer_fallback", C.c_uint64),
        ("defer_redo_level", C.c_uint64), ("narrow_levels", C.c_uint64),
        ("claim_mode", C.c_int),
    ]


class KcSqueueConfig(C.Structure):
    _fields_ = [
        ("state_words", C.c_int), ("device", C.c_int), ("segment_states", C.c_uint64),
        ("hbm_bytes", C.c_uint64), ("host_bytes", C.c_uint64), ("spill_dir", C.c_char_p),
    ]


class KcSqueueStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "size", "segments", "seg_hbm", "seg_host", "seg_disk", "hbm_bytes", "host_bytes", "disk_bytes",
        "spilled_host_bytes", "spilled_disk_bytes", "reloaded_bytes", "peak_hbm_bytes")]


# (name, restype, argtypes) for every symbol of include/kubecheck.h
_P = C.c_void_p
_U64P = C.POINTER(C.c_uint64)

# kc_host_comm: the caller's collectives for kc_group_create_host
HC_ALL_GATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64))
HC_EXCHANGE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_int, C.c_void_p, C.c_void_p)
HC_BROADCAST = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_uint64))
HC_ALL_REDUCE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_uint64)


class KcHostComm(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("all_gather", HC_ALL_GATHER), ("exchange", HC_EXCHANGE),
                ("broadcast", HC_BROADCAST), ("all_reduce_sum", HC_ALL_REDUCE)]

_U8P = C.POINTER(C.c_uint8)
_IP = C.POINTER(C.c_int)
SIGNATURES = [
    ("kc_last_error", C.c_char_p, []),
    ("kc_abi_version", C.c_int, []),
    ("kc_build_info", C.c_char_p, []),
    ("kc_device_count", C.c_int, []),
    ("kc_fpset_create", C.c_int, [C.c_uint64, C.c_int, C.POINTER(_P)]),
    ("kc_fpset_destroy", None, [_P]),
    ("kc_fpset_put_batch", C.c_int, [_P, _U64P, C.c_size_t, _U8P]),
    ("kc_fpset_contains_batch", C.c_int, [_P, _U64P, C.c_size_t, _U8P]),
    ("kc_fpset_put_batch_dev", C.c_int, [_P, _P, C.c_size_t, _P, _P]),
    ("kc_fpset_contains_batch_dev", C.c_int, [_P, _P, C.c_size_t, _P, _P]),
    ("kc_fpset_size", C.c_uint64, [_P]),
    ("kc_fpset_capacity", C.c_uint64, [_P]),
    ("kc_fpset_check_fps", C.c_int, [_P, _U64P, C.POINTER(C.c_double)]),
    ("kc_fpset_stress", C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                  C.POINTER(C.c_double), C.POINTER(C.c_double), _U64P]),
    ("kc_fpset_put", C.c_int, [_P, C.c_uint64, _IP]),
    ("kc_fpset_contains", C.c_int, [_P, C.c_uint64, _IP]),
    ("kc_fpset_combine_rounds", C.c_uint64, [_P]),
    ("kc_fpset_insert_count_dev", C.c_int, [_P, _P, C.c_size_t, _U64P, _P]),
    ("kc_fpset_contains_count_dev", C.c_int, [_P, _P, C.c_size_t, _U64P, _P]),
    ("kc_fpset_partition_dev", C.c_int, [_P, _P, C.c_uint64, C.c_int, _P, _U64P, _P]),
    ("kc_stress_fps_dev", C.c_int, [C.c_uint64, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, _P, _P]),
    ("kc_stress_fp", C.c_uint64, [C.c_uint64, C.c_int, C.c_uint64, C.c_uint64]),
    ("kc_squeue_create", C.c_int, [C.c_int, C.c_uint64, C.c_int, C.POINTER(_P)]),
    ("kc_squeue_create2", C.c_int, [C.POINTER(KcSqueueConfig), C.POINTER(_P)]),
    ("kc_squeue_enqueue_dev", C.c_int, [_P, _P, C.c_size_t, _P]),
    ("kc_squeue_dequeue_dev", C.c_int, [_P, _P, C.c_size_t, C.POINTER(C.c_size_t), _P]),
    ("kc_squeue_reserve_dev", C.c_int, [_P, C.c_size_t, C.POINTER(_P), _P]),
    ("kc_squeue_commit", C.c_int, [_P, C.c_size_t, _P]),
    ("kc_squeue_front_dev", C.c_int, [_P, C.c_size_t, C.c_size_t, C.POINTER(_P), C.POINTER(C.c_size_t), _P]),
    ("kc_squeue_pop", C.c_int, [_P, C.c_size_t, _P]),
    ("kc_squeue_peek", C.c_int, [_P, C.c_size_t, C.c_size_t, _U64P, _P]),
    ("kc_squeue_get_stats", C.c_int, [_P, C.POINTER(KcSqueueStats)]),
    ("kc_squeue_destroy", None, [_P]),
    ("kc_squeue_enqueue", C.c_int, [_P, _U64P, C.c_size_t]),
    ("kc_squeue_dequeue", C.c_int, [_P, _U64P, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("kc_squeue_size", C.c_uint64, [_P]),
    ("kc_model_config_default", None, [C.POINTER(KcModelConfig)]),
    ("kc_engine_create", C.c_int, [C.POINTER(KcModelConfig), C.POINTER(_P)]),
    ("kc_engine_destroy", None, [_P]),
    ("kc_engine_run", C.c_int, [_P, C.POINTER(KcResult)]),
    ("kc_engine_trace_text", C.c_size_t, [_P, C.c_char_p, C.c_size_t]),
    ("kc_engine_trace_tuple", C.c_int, [_P, C.c_int, _U64P]),
    ("kc_engine_level_tuples", C.c_int64, [_P, C.c_int, _U64P, C.c_uint64]),
    ("kc_engine_capture_level", C.c_int, [_P, C.c_int]),
    ("kc_engine_kernel_times", C.c_int, [_P, C.POINTER(C.c_double), _U64P]),
    ("kc_engine_narrow_times", C.c_int, [_P, C.POINTER(C.c_double), _U64P, _U64P]),
    ("kc_engine_check_fps", C.c_int, [_P, _U64P, C.POINTER(C.c_double)]),
    ("kc_shard_create", C.c_int, [C.POINTER(KcModelConfig), C.c_int, C.c_int, C.POINTER(_P)]),
    ("kc_shard_destroy", None, [_P]),
    ("kc_shard_init", C.c_int, [_P, _U64P]),
    ("kc_shard_init_error", C.c_int, [_P, _U64P]),
    ("kc_shard_set_stream", C.c_int, [_P, _P]),
    ("kc_shard_expand", C.c_int, [_P, _U64P, _U64P]),
    ("kc_shard_record_bytes", C.c_uint64, [_P]),
    ("kc_shard_pack", C.c_int, [_P, _P]),
    ("kc_shard_insert", C.c_int, [_P, _P, C.c_uint64, _U64P, _U64P]),
    ("kc_shard_advance", C.c_int, [_P]),
    ("kc_shard_parent_key", C.c_int, [_P, C.c_int, C.c_uint64, _U64P]),
    ("kc_shard_frontier_tuple", C.c_int, [_P, C.c_uint64, _U64P]),
    ("kc_shard_result", C.c_int, [_P, C.POINTER(KcResult)]),
    ("kc_shard_claim_times", C.c_int, [_P, C.POINTER(C.c_double), _U64P, _U64P]),
    ("kc_shard_owner", C.c_int, [C.c_uint64, C.c_int]),
    ("kc_rccl_unique_id", C.c_int, [C.c_char_p]),
    ("kc_group_create_rccl", C.c_int, [_P, C.c_char_p, C.POINTER(_P)]),
    ("kc_group_create_local", C.c_int, [C.POINTER(_P), C.c_int, C.POINTER(_P)]),
    ("kc_group_create_host", C.c_int, [_P, C.POINTER(KcHostComm), C.POINTER(_P)]),
    ("kc_group_destroy", None, [_P]),
    ("kc_group_run", C.c_int, [_P, C.POINTER(KcResult)]),
    ("kc_group_trace_tuple", C.c_int, [_P, C.c_int, _U64P]),
    ("kc_group_records_sent", C.c_uint64, [_P]),
    ("kc_exchange_plan", C.c_int, [C.c_int, C.c_int, _U64P, C.c_uint64, _U64P, C.c_int]),
    ("kc_cold_find_selftest", C.c_int64, [C.c_uint64, C.c_uint64]),
    ("kc_spec_tuple_words", C.c_int, [C.c_int, C.c_int, C.c_int]),
    ("kc_spec_state_words", C.c_int, [C.c_int, C.c_int, C.c_int]),
    ("kc_spec_init", C.c_int, [C.POINTER(KcModelConfig), _U64P, C.c_int]),
    ("kc_spec_successors", C.c_int, [C.POINTER(KcModelConfig), _U64P, _IP, _U64P, C.c_int, _IP]),
    ("kc_spec_check", C.c_int, [C.POINTER(KcModelConfig), _U64P]),
    ("kc_spec_fingerprint", C.c_int, [C.POINTER(KcModelConfig), _U64P, _U64P]),
    ("kc_spec_fp_selfcheck", C.c_int, [C.POINTER(KcModelConfig), _U64P]),
    ("kc_spec_pack", C.c_int, [C.POINTER(KcModelConfig), _U64P, _U64P]),
    ("kc_spec_unpack", C.c_int, [C.POINTER(KcModelConfig), _U64P, _U64P]),
]

_lib = None


class KubecheckError(RuntimeError):
    def __init__(self, func: str, code: int, msg: str):
        super().__init__(f"{func} failed ({code}): {msg}")
        self.code = code


def load() -> C.CDLL:
    """Load libkubecheck.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 and
    # cannot initialise on top of /opt/rocm's if that one is loaded first, so
    # when torch is installed it is loaded before libkubecheck (whose
    # libamdhip64.so.7 dependency then resolves to the already-loaded copy).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libkubecheck.so not found at {LIB_PATH}; build it with "
            "`make -C tla-kubernetes_amd/csrc` (or __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def build_id() -> str:
    """A digest of the HIP sources libkubecheck.so is built from (csrc/*.hip,
    *.h and the C-ABI header).  Profiles record it (tools/pmc_summary.py), so
    a bench line uses a committed PMC figure as a measurement only when it
    was taken on the kernels of this build."""
    import hashlib
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
    hdr = os.path.join(os.path.dirname(os.path.dirname(csrc)), "include", "kubecheck.h")
    h = hashlib.sha1()
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h"))) if os.path.isdir(csrc) else []
    for f in [os.path.join(csrc, f) for f in files] + [hdr]:
        try:
            with open(f, "rb") as fh:
                h.update(os.path.basename(f).encode() + b"\0" + fh.read())
        except OSError:
            pass
    return h.hexdigest()[:16]


def check(func: str, rc: int) -> int:
    if rc < 0:
        msg = load().kc_last_error()
        raise KubecheckError(func, rc, msg.decode() if msg else "")
    return rc
