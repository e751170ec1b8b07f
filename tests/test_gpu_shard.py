"""HIP shard stages (kc_shard_*) on one GPU: R ranks emulated in one process
by exchanging the device send buffers directly (the box has one GPU; RCCL
needs one process per GPU).  Counts, widths, per-action generated counts
and error traces must equal the single-GPU/oracle results for every R.
Also runs the real driver (RCCL via torch.distributed) at world_size 1."""
import os
import socket

import numpy as np
import pytest
import torch

from kubecheck import ACTIONS, ModelConfig, Spec
from kubecheck.distributed import HipShard, NONE_KEY

pytestmark = pytest.mark.gpu


def emulate(R, **kw):
    cfg = ModelConfig(**kw)
    shards = [HipShard(cfg, r, R) for r in range(R)]
    rb = shards[0].record_bytes
    n = sum(s.init() for s in shards)
    widths, err = [n], NONE_KEY
    while True:
        sends, counts = [], []
        init_err = NONE_KEY
        for s in shards:
            c, e = s.expand()
            if (e & 0xFF) == 0x12 and e != NONE_KEY:
                init_err = min(init_err, e)       # Init violations precede level-2 errors
            err = min(err, e)
            buf = torch.empty(max(sum(c), 1) * rb // 8, dtype=torch.int64, device="cuda")
            s.pack(buf)
            sends.append(buf)
            counts.append(c)
        if init_err != NONE_KEY:
            err = init_err
            break
        total = 0
        for r, s in enumerate(shards):
            parts, m = [], 0
            for src in range(R):
                off = sum(counts[src][:r]) * rb // 8
                parts.append(sends[src][off: off + counts[src][r] * rb // 8])
                m += counts[src][r]
            recv = torch.cat(parts) if m else torch.empty(rb // 8, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            nn, e = s.insert(recv, m)
            err = min(err, e)
            total += nn
        if err != NONE_KEY or total == 0:
            break
        for s in shards:
            s.advance()
        widths.append(total)
    res = [s.result() for s in shards]
    out = {"level_width": widths, "err": err,
           "distinct": sum(r["distinct"] for r in res),
           "generated": sum(r["init"] + r["generated"] for r in res),
           "act_gen": dict(zip(ACTIONS, np.sum([r["act_gen"] for r in res], axis=0).tolist()))}
    for s in shards:
        s.close()
    return out


@pytest.mark.parametrize("R", [1, 2, 4, 8])
def test_model1_any_shard_count(fixtures, R):
    fx = fixtures["model1"]
    r = emulate(R)
    assert r["err"] == NONE_KEY
    assert r["level_width"] == fx["level_width"]
    assert (r["distinct"], r["generated"]) == (fx["distinct"], fx["generated"])
    assert r["act_gen"] == fx["act_gen"]


@pytest.mark.parametrize("R", [2, 3, 9])
def test_errors_sharded(fixtures, R):
    # R = 9: error keys of ranks >= 8 are >= 2^63
    r = emulate(R, nc=2)
    assert r["err"] & 0xFF == 1 and len(r["level_width"]) == 10
    assert r["level_width"] == fixtures["nc2"]["level_width"]
    r = emulate(R, variant=2)
    assert r["err"] & 0xFF == 2
    assert len(r["level_width"]) + 1 == fixtures["variant2"]["err_level"]
    r = emulate(R, variant=3)
    assert r["err"] & 0xFF == 1 and len(r["level_width"]) == fixtures["variant3"]["err_level"]
    r = emulate(R, ns=0)
    assert r["err"] & 0xFF == 3 and len(r["level_width"]) == fixtures["ns0"]["err_level"]
    r = emulate(R, variant=5)                 # an Init state violates OnlyOneVersion
    assert r["err"] & 0xFF == 0x12 and len(r["level_width"]) == 1


def test_enlarged_prefix_sharded(fixtures):
    fx = fixtures["np2_40levels"]
    assert emulate_levels(4, 40, np=2) == fx["level_width"]


def emulate_levels(R, L, **kw):
    cfg = ModelConfig(**kw)
    shards = [HipShard(cfg, r, R) for r in range(R)]
    rb = shards[0].record_bytes
    widths = [sum(s.init() for s in shards)]
    while len(widths) < L:
        sends, counts = [], []
        for s in shards:
            c, _ = s.expand()
            buf = torch.empty(max(sum(c), 1) * rb // 8, dtype=torch.int64, device="cuda")
            s.pack(buf)
            sends.append(buf)
            counts.append(c)
        total = 0
        for r, s in enumerate(shards):
            rw = rb // 8
            parts = [sends[src][sum(counts[src][:r]) * rw: (sum(counts[src][:r]) + counts[src][r]) * rw]
                     for src in range(R)]
            m = sum(counts[src][r] for src in range(R))
            recv = torch.cat(parts)
            torch.cuda.synchronize()          # the shard reads recv on its own stream
            total += s.insert(recv, m)[0]
        for s in shards:
            s.advance()
        widths.append(total)
    for s in shards:
        s.close()
    return widths


def test_driver_world1_rccl(fixtures):
    import torch.distributed as dist
    from kubecheck.distributed import ShardedModelChecker

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        cfg = ModelConfig()
        r = ShardedModelChecker(cfg, HipShard(cfg, 0, 1)).run()
        fx = fixtures["model1"]
        assert r["level_width"] == fx["level_width"]
        assert (r["distinct"], r["generated"]) == (fx["distinct"], fx["generated"])
        cfg2 = ModelConfig(nc=2)
        r2 = ShardedModelChecker(cfg2, HipShard(cfg2, 0, 1)).run()
        assert r2["error"] == "assertion" and r2["trace"] == fixtures["nc2"]["trace"]
        for key, kw, kind in (("variant5", dict(variant=5), "invariant"),
                              ("ns0", dict(ns=0), "deadlock"),
                              ("variant4", dict(variant=4), "invariant")):
            c = ModelConfig(**kw)
            r3 = ShardedModelChecker(c, HipShard(c, 0, 1)).run()
            assert r3["error"] == kind and r3["trace_len"] == fixtures[key]["trace_len"]
            assert r3["error_level"] == fixtures[key]["err_level"]
    finally:
        dist.destroy_process_group()


# --- the native level loop (kc_group_*): the same protocol in C++ --------
from kubecheck.distributed import NativeShardedChecker


def native(R, **kw):
    mc = NativeShardedChecker(ModelConfig(**kw), emulate=R)
    try:
        return mc.run()
    finally:
        mc.close()


@pytest.mark.parametrize("R", [1, 2, 3, 8, 9])
def test_native_model1_any_rank_count(fixtures, R):
    fx = fixtures["model1"]
    r = native(R)
    assert r["complete"] and r["error"] is None
    assert r["level_width"] == fx["level_width"]
    assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r["act_gen"] == fx["act_gen"]
    assert sum(r["act_dist"].values()) + r["init"] == r["distinct"]


@pytest.mark.parametrize("R", [2, 9])
@pytest.mark.parametrize("key,kw,kind", [("nc2", dict(nc=2), "assertion"),
                                         ("variant2", dict(variant=2), "invariant"),
                                         ("variant3", dict(variant=3), "assertion"),
                                         ("variant5", dict(variant=5), "invariant"),
                                         ("ns0", dict(ns=0), "deadlock")])
def test_native_error_paths(fixtures, oracle, R, key, kw, kind):
    fx = fixtures[key]
    r = native(R, **kw)
    assert r["error"] == kind
    assert (r["error_level"], r["trace_len"]) == (fx["err_level"], fx["trace_len"])
    if kind == "assertion":
        assert r["error_action"] == fx["err_action"]
    # the trace is a real behaviour from an Init state, ending in the error
    # (with R > 1 ranks the frontier order differs, so when a level holds
    # several errors an equally short one may be reported)
    cfg = oracle.config(nc=kw.get("nc", 1), ns=kw.get("ns", 1), variant=kw.get("variant", 0))
    for a, b in zip(r["trace"], r["trace"][1:]):
        succ, _ = oracle.successors(cfg, a)
        assert any(list(map(int, x)) == b for _, x in succ)


def test_native_enlarged_prefix(fixtures):
    fx = fixtures["np2_40levels"]
    r = native(4, np=2, max_levels=40)
    assert r["level_width"] == fx["level_width"] and not r["complete"]
    assert r["act_gen"] == fx["act_gen"]


@pytest.mark.parametrize("devrow", ["1", "0"])
def test_native_rccl_world1(fixtures, monkeypatch, devrow):
    # the RCCL communicator path (one rank: every collective runs, nothing
    # moves; KC_RCCL_FORCE=1 keeps the world-1 collectives on RCCL), with the
    # all-gather row written by the shard's kernels in device memory (the
    # N-GPU default) and with host rows (KC_DEVROW=0)
    monkeypatch.setenv("KC_RCCL_FORCE", "1")
    monkeypatch.setenv("KC_DEVROW", devrow)
    for key, kw, kind in (("variant5", dict(variant=5), "invariant"),   # Init state: key 0x12
                          ("ns0", dict(ns=0), "deadlock"),
                          ("variant3", dict(variant=3), "assertion")):
        mc = NativeShardedChecker(ModelConfig(**kw), 0, 1)
        try:
            r = mc.run()
            assert r["error"] == kind
            assert (r["error_level"], r["trace_len"]) == (fixtures[key]["err_level"], fixtures[key]["trace_len"])
        finally:
            mc.close()
    mc = NativeShardedChecker(ModelConfig(), 0, 1)
    try:
        r = mc.run()
        fx = fixtures["model1"]
        assert r["level_width"] == fx["level_width"]
        assert (r["distinct"], r["generated"]) == (fx["distinct"], fx["generated"])
    finally:
        mc.close()
    mc = NativeShardedChecker(ModelConfig(nc=2), 0, 1)
    try:
        r = mc.run()
        assert r["error"] == "assertion" and r["trace"] == fixtures["nc2"]["trace"]
    finally:
        mc.close()


@pytest.mark.parametrize("R", [8])
def test_native_enlarged_full_emulated(fixtures, R):
    # the whole NP=2 model through the native sharded loop with 8 ranks on one
    # GPU (LocalComm): the 8-GPU protocol at full size, against the golden
    fx = fixtures["np2_full"]
    mc = NativeShardedChecker(ModelConfig(np=2, keep_trace=False), emulate=R)
    try:
        r = mc.run()
    finally:
        mc.close()
    assert r["complete"] and r["error"] is None
    assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r["level_width"] == fx["level_width"]
    assert r["act_gen"] == fx["act_gen"]


def test_native_np3_47_levels_emulated():
    # NP=3 (the scaling workload's model) through the native sharded loop with
    # 4 ranks on one GPU: its first 47 levels, 341,685,569 states, against the
    # widths of the oracle's 128-bit multi-threaded BFS (np3_52levels.json).
    # (All 52 levels, 1.09e9 states, need more HBM than four ranks' buffers
    # get on one GPU; the engine checks them, test_gpu_engine.py.)
    import json
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "np3_52levels.json")))
    mc = NativeShardedChecker(ModelConfig(np=3, max_levels=47, keep_trace=False), emulate=4)
    try:
        r = mc.run()
    finally:
        mc.close()
    assert r["error"] is None and not r["complete"] and r["depth"] == 47
    assert r["level_width"] == fx["level_width"][:47]
    assert r["distinct"] == sum(fx["level_width"][:47]) == 341685569


def test_native_multipiece_emulated(fixtures, monkeypatch):
    # the exchange cut into pieces of 85 records (KC_PIECE_BYTES=4096; the
    # N-GPU default is 256 MiB): the emulated ranks replay every rank's
    # RCCL plan (kc_exchange_plan) piece by piece, exact against the golden
    monkeypatch.setenv("KC_PIECE_BYTES", "4096")
    fx = fixtures["model1"]
    r = native(3)
    assert r["level_width"] == fx["level_width"]
    assert (r["distinct"], r["generated"]) == (fx["distinct"], fx["generated"])
    fx = fixtures["np2_40levels"]
    r = native(5, np=2, max_levels=40)
    assert r["level_width"] == fx["level_width"] and r["act_gen"] == fx["act_gen"]


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
@pytest.mark.parametrize("devrow", ["1", "0"])
def test_native_fault_stops_every_rank(monkeypatch, stage, devrow):
    # a failure on one rank (KC_FAULT=rank:level:stage) travels in the
    # all-gather row: every rank leaves the loop with an error at the next
    # gather instead of waiting in a collective for the failed one
    from kubecheck import KubecheckError
    monkeypatch.setenv("KC_DEVROW", devrow)
    monkeypatch.setenv("KC_FAULT", f"2:7:{stage}")
    with pytest.raises(KubecheckError) as e:
        native(4)
    assert "injected fault" in str(e.value) and e.value.code == -5
    monkeypatch.setenv("KC_FAULT", f"0:7:{stage}")
    monkeypatch.setenv("KC_RCCL_FORCE", "1")
    mc = NativeShardedChecker(ModelConfig(), 0, 1)
    try:
        with pytest.raises(KubecheckError) as e:
            mc.run()
        assert "injected fault" in str(e.value)
    finally:
        mc.close()


@pytest.mark.parametrize("R", [1, 2, 3])
def test_native_lost_update_invariant(fixtures, R):
    # NoLostUpdate (build-defined; variant 1 = Update without HasRead) through
    # the sharded loop: same error, level and trace length as the oracle
    fx = fixtures["variant1_lost_update"]
    r = native(R, variant=1, invariants=7)
    assert r["error"] == "invariant" and r["error_invariant"] == "NoLostUpdate"
    assert (r["error_level"], r["trace_len"]) == (fx["err_level"], fx["trace_len"])
    if R == 1:
        assert r["trace"] == fx["trace"]


@pytest.mark.parametrize("R", [2, 3, 9])
def test_native_init_violation_tlc_order(fixtures, R):
    # variant 5: EVERY Init state violates OnlyOneVersion; the one reported
    # is the first in TLC's Init order whichever rank owns it,
    # the same state the oracle and the single-GPU engine report
    fx = fixtures["variant5"]
    r = native(R, variant=5)
    assert r["error"] == "invariant" and r["error_level"] == 1
    assert r["trace"] == fx["trace"]


@pytest.mark.parametrize("R", [1, 3])
def test_native_init_violation_max_levels_1(fixtures, R):
    # an Init state's invariant violation (variant 5) is level 1's error even
    # when level 1 is never expanded
    r = native(R, variant=5, max_levels=1)
    assert r["error"] == "invariant" and r["error_level"] == 1 and r["trace_len"] == 1


# --- round 5: record staging and the deferred frontier on the counted path
@pytest.mark.parametrize("R", [1, 2, 3])
def test_native_counted_deferred(fixtures, monkeypatch, R):
    # KC_SNARROW=0: every level on the counted path, so every level after the
    # first runs on a deferred frontier (links only; the next expand rebuilds
    # the states and finds their invariant violations there) and, with R > 1,
    # packs its records through the tiles' staging segments
    monkeypatch.setenv("KC_SNARROW", "0")
    fx = fixtures["model1"]
    r = native(R)
    assert r["level_width"] == fx["level_width"]
    assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r["act_gen"] == fx["act_gen"]
    # (per-action distinct counts follow each state's first discoverer: TLC's
    # at R = 1; at R > 1 the rank-major claim order picks another copy)
    if R == 1:
        assert r["act_dist"] == fx["act_dist"]
    assert sum(r["act_dist"].values()) + r["init"] == r["distinct"]
    for key, kw, kind in (("nc2", dict(nc=2), "assertion"), ("variant2", dict(variant=2), "invariant"),
                          ("variant3", dict(variant=3), "assertion"), ("ns0", dict(ns=0), "deadlock"),
                          ("variant4", dict(variant=4), "invariant"),
                          ("variant1_lost_update", dict(variant=1, invariants=7), "invariant")):
        fk = fixtures[key]
        r = native(R, **kw)
        assert r["error"] == kind, key
        assert (r["error_level"], r["trace_len"]) == (fk["err_level"], fk["trace_len"]), key
        if R == 1:
            assert r["trace"] == fk["trace"], key


@pytest.mark.parametrize("R", [1, 3])
def test_native_np2_lost_update_deferred(fixtures, R):
    # NP=2's NoLostUpdate violation at depth 25 is found on a wide (counted,
    # deferred) level: as the next expand rebuilds level 25's states
    fk = fixtures["np2_variant1_lost_update"]
    r = native(R, np=2, variant=1, invariants=7)
    assert r["error"] == "invariant" and r["error_invariant"] == "NoLostUpdate"
    assert (r["error_level"], r["trace_len"]) == (fk["err_level"], fk["trace_len"])
    if R == 1:
        assert r["trace"] == fk["trace"]


# --- round 5: TLC-ordered claims at R > 1 (ModelConfig.tlc_order)
TLC_CASES = (("nc2", dict(nc=2), "assertion"), ("variant2", dict(variant=2), "invariant"),
             ("variant3", dict(variant=3), "assertion"), ("ns0", dict(ns=0), "deadlock"),
             ("variant4", dict(variant=4), "invariant"),
             ("variant1_lost_update", dict(variant=1, invariants=7), "invariant"))


@pytest.mark.parametrize("R", [2, 3, 9])
def test_native_tlc_order(fixtures, R):
    # claims ordered by the parents' sequential-BFS positions: every state's
    # first discoverer is TLC -workers 1's, so the per-action distinct counts
    # and every counterexample trace equal the oracle's state for state
    fx = fixtures["model1"]
    r = native(R, tlc_order=True)
    assert r["complete"] and r["level_width"] == fx["level_width"]
    assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r["act_gen"] == fx["act_gen"] and r["act_dist"] == fx["act_dist"]
    for key, kw, kind in TLC_CASES:
        fk = fixtures[key]
        r = native(R, tlc_order=True, **kw)
        assert r["error"] == kind, key
        assert (r["error_level"], r["trace_len"]) == (fk["err_level"], fk["trace_len"]), key
        assert r["trace"] == fk["trace"], key
        if kind == "assertion":
            assert r["error_action"] == fk["err_action"], key


def test_native_tlc_order_np2(fixtures):
    # NP=2's NoLostUpdate violation at depth 25 (wide levels) and the 40-level
    # prefix, TLC-ordered at 3 and 4 ranks
    fk = fixtures["np2_variant1_lost_update"]
    r = native(3, np=2, variant=1, invariants=7, tlc_order=True)
    assert r["error"] == "invariant" and r["error_invariant"] == "NoLostUpdate"
    assert (r["error_level"], r["trace_len"]) == (fk["err_level"], fk["trace_len"])
    assert r["trace"] == fk["trace"]
    fx = fixtures["np2_40levels"]
    r = native(4, np=2, max_levels=40, tlc_order=True)
    assert r["level_width"] == fx["level_width"] and r["act_gen"] == fx["act_gen"]


def test_native_np2_prefix_switches(fixtures, monkeypatch):
    # the NP=2 40-level prefix at 4 emulated ranks with each round-5 path
    # switched off in turn (materialising emit, k_shard_pack, per-parent
    # scans): counts equal to the oracle's, and every per-action distinct
    # count equal across the variants (the same claims win whichever path
    # built, packed or positioned the states)
    fx = fixtures["np2_40levels"]
    runs = {}
    for name, env in (("default", {}), ("sdefer0", {"KC_SDEFER": "0"}), ("stage0", {"KC_STAGE": "0"}),
                      ("tscan0", {"KC_SHARD_TSCAN": "0"})):
        for k in ("KC_SDEFER", "KC_STAGE", "KC_SHARD_TSCAN"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        mc = NativeShardedChecker(ModelConfig(np=2, max_levels=40), emulate=4)
        try:
            r = mc.run()
            r["records_sent"] = mc.records_sent
        finally:
            mc.close()
        assert r["level_width"] == fx["level_width"] and not r["complete"], name
        assert r["act_gen"] == fx["act_gen"] and r["distinct"] == fx["distinct"], name
        runs[name] = r
    for name, r in runs.items():
        assert r["act_dist"] == runs["sdefer0"]["act_dist"], name
        assert r["records_sent"] == runs["sdefer0"]["records_sent"], name


# --- round 6: first-claim mode on the sharded loop (ModelConfig.first_claim;
# VERDICT r5 item 1): a state belongs to the copy whose ClaimSet CAS inserts
# it, as in a TLC -workers N run — no candidates, no settle passes, the
# records' claims CAS-only.  Counts, widths, depth, per-action generated
# counts, error kinds, levels and trace lengths are the deterministic mode's;
# which same-level copy wins is not (so per-action distinct counts and the
# trace states are checked for consistency, not equality).
FIRST_CASES = TLC_CASES + (("variant5", dict(variant=5), "invariant"),)


def _first_trace_ok(oracle, kw, trace):
    cfg = oracle.config(nc=kw.get("nc", 1), ns=kw.get("ns", 1), variant=kw.get("variant", 0),
                        invariants=kw.get("invariants", 3))
    init = {tuple(map(int, t)) for t in oracle.level_tuples(cfg, 1)}
    assert tuple(trace[0]) in init
    for a, b in zip(trace, trace[1:]):
        succ, _ = oracle.successors(cfg, a)
        assert any(list(map(int, x)) == b for _, x in succ)


@pytest.mark.parametrize("R", [1, 2, 3, 8])
@pytest.mark.parametrize("snarrow", ["1", "0"])
def test_native_first_claim(fixtures, oracle, monkeypatch, R, snarrow):
    # snarrow 0: every level on the counted path (every claim first-claim)
    monkeypatch.setenv("KC_SNARROW", snarrow)
    fx = fixtures["model1"]
    r = native(R, first_claim=True)
    assert r["claim_mode"] == "first"
    assert r["complete"] and r["error"] is None and r["level_width"] == fx["level_width"]
    assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r["act_gen"] == fx["act_gen"]
    assert sum(r["act_dist"].values()) + r["init"] == r["distinct"]
    for key, kw, kind in FIRST_CASES:
        fk = fixtures[key]
        r = native(R, first_claim=True, **kw)
        assert r["error"] == kind, key
        assert (r["error_level"], r["trace_len"]) == (fk["err_level"], fk["trace_len"]), key
        if kind == "assertion":
            assert r["error_action"] == fk["err_action"], key
        _first_trace_ok(oracle, kw, r["trace"])


@pytest.mark.parametrize("first", [True, False])
def test_native_owner_chunk_scan_off(fixtures, monkeypatch, first):
    # round 6: the staged records' positions come from owner x 64-tile chunk
    # sums (k_owner_cscan, k_shard_gather's in-chunk prefix) by default;
    # KC_CHUNK_SCAN=0 keeps the per-tile owner scan — same counts and widths
    # at R = 3 with every level counted
    monkeypatch.setenv("KC_CHUNK_SCAN", "0")
    monkeypatch.setenv("KC_SNARROW", "0")
    fx = fixtures["model1"]
    r = native(3, first_claim=first)
    assert r["complete"] and r["error"] is None and r["level_width"] == fx["level_width"]
    assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
    fx = fixtures["np2_40levels"]
    r = native(4, np=2, max_levels=40, first_claim=first)
    assert r["level_width"] == fx["level_width"] and r["act_gen"] == fx["act_gen"]


def test_native_first_claim_np2(fixtures):
    # NP=2: the 40-level prefix at 4 emulated ranks, and the seeded race's
    # NoLostUpdate violation at depth 25 (wide, deferred levels) at 3
    fx = fixtures["np2_40levels"]
    r = native(4, np=2, max_levels=40, first_claim=True)
    assert r["level_width"] == fx["level_width"] and r["act_gen"] == fx["act_gen"] and not r["complete"]
    assert r["distinct"] == fx["distinct"]
    fk = fixtures["np2_variant1_lost_update"]
    r = native(3, np=2, variant=1, invariants=7, first_claim=True)
    assert r["error"] == "invariant" and r["error_invariant"] == "NoLostUpdate"
    assert (r["error_level"], r["trace_len"]) == (fk["err_level"], fk["trace_len"])


def test_native_enlarged_full_emulated_first_claim(fixtures):
    # the whole NP=2 model at 8 emulated ranks in first-claim mode (the
    # deterministic mode's run is test_native_enlarged_full_emulated), exact
    # against the golden
    fx = fixtures["np2_full"]
    mc = NativeShardedChecker(ModelConfig(np=2, keep_trace=False, first_claim=True), emulate=8)
    try:
        r = mc.run()
    finally:
        mc.close()
    assert r["claim_mode"] == "first"
    assert r["complete"] and r["error"] is None
    assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r["level_width"] == fx["level_width"] and r["act_gen"] == fx["act_gen"]


def test_native_first_claim_rejects_tlc_order():
    # first-claim and TLC order are two different claim orders
    from kubecheck import KubecheckError
    with pytest.raises(KubecheckError) as e:
        native(2, first_claim=True, tlc_order=True)
    assert "first_claim" in str(e.value) and e.value.code == -22
