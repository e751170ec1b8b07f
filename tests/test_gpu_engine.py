"""GPU engine parity: the HIP BFS (through the C-ABI) against the reference's
recorded run (MC.out) and the CPU oracle, on the same models.  Integer
counts, level widths, per-action counts, state sets and traces must be
bit-identical."""
import numpy as np
import pytest

import kubecheck
from kubecheck import ModelChecker, ModelConfig

pytestmark = pytest.mark.gpu


def run(**kw):
    with ModelChecker(ModelConfig(**kw)) as mc:
        return mc.run()


@pytest.fixture(scope="module")
def model1():
    return run()


def test_model1_matches_mcout(model1, mcout):
    r = model1
    assert (r.init, r.generated, r.distinct, r.queue_left, r.depth) == (
        mcout["init"], mcout["generated"], mcout["distinct"], mcout["queue_left"], mcout["depth"])
    assert r.complete and r.error is None
    assert r.act_gen == mcout["act_gen"]                       # MC.out:78-621
    assert f"{r.collision_optimistic:.1E}" == f"{mcout['collision_optimistic']:.1E}"


def test_model1_matches_oracle_order(model1, fixtures):
    fx = fixtures["model1"]
    assert model1.level_width == fx["level_width"]
    # per-action distinct counts follow the sequential (1-worker) BFS order
    assert model1.act_dist == fx["act_dist"]


@pytest.mark.parametrize("level", [2, 37, 51, 124])
def test_level_state_sets_identical(oracle, level):
    with ModelChecker(ModelConfig()) as mc:
        mc.capture_level(level)
        mc.run()
        got = mc.level_tuples(level)
    want = oracle.level_tuples(oracle.config(), level)
    assert got.shape == want.shape
    assert np.array_equal(got, want)          # same states, same FIFO order


@pytest.mark.parametrize("f,t", [(0, 0), (0, 1), (1, 0)])
def test_constant_variants(fixtures, f, t):
    r = run(can_fail=f, can_timeout=t)
    fx = fixtures[f"model1_fail{f}_timeout{t}"]
    assert (r.distinct, r.generated, r.depth) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r.level_width == fx["level_width"] and r.act_gen == fx["act_gen"]


def test_multi_chunk_and_rehash_paths(model1):
    # tiny chunks (many k_count_chunks/expand/resolve/emit rounds per level) and
    # a tiny initial FPSet (repeated rehash) must not change anything
    r = run(chunk_states=256, fpset_slots=64)
    assert (r.distinct, r.generated, r.depth) == (model1.distinct, model1.generated, model1.depth)
    assert r.level_width == model1.level_width
    assert r.act_gen == model1.act_gen and r.act_dist == model1.act_dist
    assert r.fpset_slots > 64


@pytest.mark.parametrize("env", [{"KC_TSCAN_REG": "0"}, {"KC_TSCAN": "0", "KC_DEFER": "0"}, {"KC_HEADCOPY": "1"},
                                 {"KC_DEFER": "0"}])
def test_wide_level_variants(model1, monkeypatch, env):
    # every level on the wide path (chunk_states turns the narrow kernel
    # off) with: the tile scan's loop path (levels wider than 65,536 tiles
    # take it; forced here), the per-parent hipcub scan (the materialising
    # path only: the deferred emit takes tile offsets), the copy + reset
    # read-back of the level head, and the materialising emit (KC_DEFER=0)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    r = run(chunk_states=1 << 20)
    assert (r.distinct, r.generated, r.depth) == (model1.distinct, model1.generated, model1.depth)
    assert r.level_width == model1.level_width
    assert r.act_gen == model1.act_gen and r.act_dist == model1.act_dist
    assert r.outdeg_hist == model1.outdeg_hist


def test_seeded_assertion_bug_trace(fixtures):
    # NC=2 clients sharing Secret/foo: C4 Assert (KubeAPI.tla:639-640) fails at depth 10
    fx = fixtures["nc2"]
    with ModelChecker(ModelConfig(nc=2)) as mc:
        r = mc.run()
    assert r.error == "assertion" and r.error_action == "C4" and r.error_level == 10
    assert r.trace_len == fx["trace_len"] == 10
    assert r.level_width == fx["level_width"]
    assert [list(map(int, t)) for t in r.trace] == fx["trace"]   # the same shortest trace
    assert "State 10:" in r.trace_text and "Client2" in r.trace_text


def test_seeded_invariant_bug_trace(fixtures):
    # variant 2: Force adds without replacing -> OnlyOneVersion (KubeAPI.tla:787) fails
    fx = fixtures["variant2"]
    with ModelChecker(ModelConfig(variant=2)) as mc:
        r = mc.run()
    assert r.error == "invariant" and r.error_invariant == "OnlyOneVersion"
    assert r.trace_len == fx["trace_len"] and r.error_level == fx["err_level"]
    assert [list(map(int, t)) for t in r.trace] == fx["trace"]


@pytest.mark.parametrize("key,kw", [("nc2_np0", dict(nc=2, np=0)), ("ns2", dict(ns=2)),
                                    ("nc1_np0", dict(np=0)), ("variant1", dict(variant=1))])
def test_other_models(fixtures, key, kw):
    fx = fixtures[key]
    r = run(**kw)
    assert (r.depth, r.level_width) == (fx["depth"], fx["level_width"])
    assert (r.error or None) == {0: None, 1: "assertion"}[fx["err_kind"]]
    if r.error is None:
        assert (r.distinct, r.generated) == (fx["distinct"], fx["generated"])
        assert r.act_gen == fx["act_gen"] and r.act_dist == fx["act_dist"]
    else:
        # a level-synchronous BFS finishes the failing level before it stops, so
        # the partial totals at an error are not comparable (TLC's are not
        # deterministic either); the error, its level and the trace are.
        assert (r.error_action, r.error_level, r.trace_len) == (
            fx["err_action"], fx["err_level"], fx["trace_len"])


def test_enlarged_prefix(fixtures):
    fx = fixtures["np2_40levels"]
    r = run(np=2, max_levels=40)
    assert r.level_width == fx["level_width"]
    assert r.act_gen == fx["act_gen"] and r.act_dist == fx["act_dist"]
    assert not r.complete


@pytest.mark.parametrize("defer", ["1", "0"])
def test_enlarged_full(fixtures, monkeypatch, defer):
    # the whole NP=2 model on the deferred frontier (links in HBM: no trace
    # store) and on the materialising path
    if "np2_full" not in fixtures:
        pytest.skip("np2_full fixture not generated")
    monkeypatch.setenv("KC_DEFER", defer)
    fx = fixtures["np2_full"]
    r = run(np=2, keep_trace=False)
    assert (r.deferred_states > 0) == (defer == "1") and not r.defer_fallback
    assert (r.distinct, r.generated, r.depth) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r.level_width == fx["level_width"]
    assert r.act_gen == fx["act_gen"] and r.act_dist == fx["act_dist"]
    assert r.complete and r.error is None


@pytest.mark.parametrize("defer", ["1", "0"])
def test_enlarged_full_first_claim(fixtures, monkeypatch, defer):
    # the bench's headline mode (round 6): the whole NP=2 model with the first
    # inserter of every state as its owner, on both frontier paths — counts,
    # depth, every level width and the per-action generated counts equal the
    # golden; the distinct split is a valid one (it sums to the new states)
    fx = fixtures["np2_full"]
    monkeypatch.setenv("KC_DEFER", defer)
    r = run(np=2, keep_trace=True, first_claim=True)
    assert r.claim_mode == "first" and not r.defer_fallback
    assert (r.distinct, r.generated, r.depth) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r.level_width == fx["level_width"] and r.act_gen == fx["act_gen"]
    assert sum(r.act_dist.values()) + r.init == r.distinct
    assert r.complete and r.error is None


# --- error paths: every kind of violation the checker
# reports, against the oracle's error, level and trace, state for state
@pytest.mark.parametrize("key,kw,kind,what", [
    ("variant3", dict(variant=3), "assertion", "C2"),          # KubeAPI.tla:598-599
    ("variant4", dict(variant=4), "invariant", "TypeOK"),      # :776-781 (IsValidListRequest)
    ("variant5", dict(variant=5), "invariant", "OnlyOneVersion"),  # an Init state (:455)
    ("ns0", dict(ns=0), "deadlock", None),                     # launch:16, no API server
])
def test_error_paths(fixtures, key, kw, kind, what):
    fx = fixtures[key]
    with ModelChecker(ModelConfig(**kw)) as mc:
        r = mc.run()
    assert r.error == kind and not r.complete
    if kind == "assertion":
        assert r.error_action == what == fx["err_action"]
    if kind == "invariant":
        assert r.error_invariant == what and fx["err_invariant"] == {"TypeOK": 0, "OnlyOneVersion": 1}[what]
    assert (r.error_level, r.trace_len) == (fx["err_level"], fx["trace_len"])
    assert [list(map(int, t)) for t in r.trace] == fx["trace"]
    # (the widths up to the error; an Init violation stops the oracle before
    # it records level 1, the engine after)
    k = min(len(r.level_width), len(fx["level_width"]))
    assert r.level_width[:k] == fx["level_width"][:k]


def test_error_without_trace_store():
    # keep_trace=False (no parent pointers): the violation is still reported
    with ModelChecker(ModelConfig(variant=3, keep_trace=False)) as mc:
        r = mc.run()
    assert r.error == "assertion" and r.error_action == "C2" and r.error_level == 23
    assert r.trace_len == 0 and r.trace == []


@pytest.mark.parametrize("key,kw", [("ns0_nodeadlock", dict(ns=0, check_deadlock=False)),
                                    ("variant4_oov_only", dict(variant=4, invariants=2)),
                                    ("variant5_no_invariants", dict(variant=5, invariants=0))])
def test_config_switches(fixtures, key, kw):
    # -deadlock and the .cfg INVARIANT list: unlisted checks are not reported
    fx = fixtures[key]
    r = run(**kw)
    assert r.complete and r.error is None
    assert (r.distinct, r.generated, r.depth) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r.level_width == fx["level_width"] and r.act_gen == fx["act_gen"]


@pytest.mark.parametrize("key,kw", [("model1", {}), ("np2_40levels", dict(np=2, max_levels=40)),
                                    ("model1_fail0_timeout0", dict(can_fail=0, can_timeout=0)),
                                    ("nc2_np0", dict(nc=2, np=0))])
def test_outdegree_histogram(fixtures, key, kw):
    # TLC's outdegree (msg 2268, MC.out:1104) = new states first reached from
    # each expanded state; under sequential BFS order it is exactly the
    # oracle's histogram (the wide and the narrow level paths both count it)
    fx = fixtures[key]
    r = run(**kw)
    if r.error is None:
        assert r.outdeg_hist == fx["outdeg_hist"]


def test_check_fps_min_gap():
    with ModelChecker(ModelConfig()) as mc:
        mc.run()
        gap, prob = mc.check_fps()
    # 163,408 fingerprints spread over [1, 2^63): the minimum gap is far below
    # the mean spacing and far above 0 (TLC reports 9.9E-10, MC.out:42)
    assert 0 < gap < 2**63 // 163408 and prob == pytest.approx(1 / gap)


# --- the resourceVersion race as an INVARIANT bug (BASELINE configs[4],
# SURVEY §8(d) config 5's second variant): variant 1 drops HasRead from
# Update (KubeAPI.tla:733), and the build-defined NoLostUpdate (invariants
# bit 2, with its lostUpdate history variable) catches the lost update
@pytest.mark.parametrize("key,kw", [("variant1_lost_update", dict(variant=1)),
                                    ("np2_variant1_lost_update", dict(np=2, variant=1))])
@pytest.mark.parametrize("mode", ["hbm", "frontier_spill", "seen_spill", "chunked"])
def test_lost_update_invariant(fixtures, key, kw, mode):
    fx = fixtures[key]
    extra = {"hbm": {}, "frontier_spill": dict(frontier_hbm_bytes=32 << 10, frontier_segment_states=256),
             "seen_spill": dict(seen_hbm_bytes=4 << 20), "chunked": dict(chunk_states=512)}[mode]
    with ModelChecker(ModelConfig(invariants=7, **kw, **extra)) as mc:
        r = mc.run()
    assert r.error == "invariant" and r.error_invariant == "NoLostUpdate" and fx["err_invariant"] == 2
    assert (r.error_level, r.trace_len) == (fx["err_level"], fx["trace_len"])
    assert [list(map(int, t)) for t in r.trace] == fx["trace"]
    assert "lostUpdate = TRUE" in r.trace_text.split("State %d:" % r.trace_len)[1]
    k = min(len(r.level_width), len(fx["level_width"]))
    assert r.level_width[:k] == fx["level_width"][:k]


def test_lost_update_holds_as_written(fixtures):
    # KubeAPI.tla as written keeps NoLostUpdate, and checking it (the ghost
    # present) leaves Model_1's state space exactly as MC.out has it
    fx = fixtures["model1_lost_update_checked"]
    r = run(invariants=7)
    assert r.complete and r.error is None
    assert (r.distinct, r.generated, r.depth) == (fx["distinct"], fx["generated"], fx["depth"]) == (
        163408, 577736, 124)
    assert r.act_dist == fx["act_dist"]


def test_np3_prefix(fixtures):
    # SURVEY §8(d) config 2's secondary model, NP=3 (4 actors: 80-B states,
    # |U| = 64): its first 40 levels (50.8M states) against the oracle
    fx = fixtures["np3_40levels"]
    r = run(np=3, max_levels=40, keep_trace=False)
    assert r.level_width == fx["level_width"]
    assert r.act_gen == fx["act_gen"] and r.act_dist == fx["act_dist"]
    assert (r.distinct, r.generated) == (fx["distinct"], fx["generated"]) and not r.complete


def test_np3_52_levels():
    # the scaling-sized workload (bench.py --workload np3_52): NP=3's first 52
    # levels, 1.1e9 states, against the oracle's multi-threaded BFS with
    # 128-bit keys (tools/np3_golden.sh; its first 40 levels equal the
    # sequential oracle's np3_40levels)
    import json
    import os
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "np3_52levels.json")))
    assert fx["fp_bits"] == 128 and fx["max_levels"] == 52 and not fx["set_full"]
    r = run(np=3, max_levels=52, keep_trace=False)
    assert r.level_width == fx["level_width"]
    assert (r.distinct, r.generated, r.depth) == (fx["distinct"], fx["generated"], fx["depth"]) == (
        r.distinct, r.generated, 52)
    assert not r.complete and r.error is None


# --- deferred frontier (engine_kernels.h DeferArgs): the wide levels' new
# states are built inside the next level's k_claim from their links
@pytest.mark.parametrize("defer", ["1", "0"])
def test_deferred_frontier_exact(fixtures, monkeypatch, defer):
    monkeypatch.setenv("KC_DEFER", defer)
    fx = fixtures["np2_40levels"]
    r = run(np=2, max_levels=40)          # keep_trace: the links are the trace entries
    assert r.level_width == fx["level_width"]
    assert r.act_gen == fx["act_gen"] and r.act_dist == fx["act_dist"]
    assert r.outdeg_hist == fx["outdeg_hist"]
    assert (r.deferred_states > 0) == (defer == "1") and not r.defer_fallback


def test_deferred_capacity_estimate_redo(fixtures, monkeypatch):
    # capacity estimates far too small (KC_DEFER_SLACK): the link buffer
    # (sized by the estimate; no trace store) overflows its guard and the run
    # is redone on the exact path
    monkeypatch.setenv("KC_DEFER_SLACK", "0.001")
    fx = fixtures["np2_40levels"]
    r = run(np=2, max_levels=40, keep_trace=False)
    # each level past its estimate is redone from that level (not from Init)
    assert r.defer_fallback and r.defer_redo_level > 1
    assert r.level_width == fx["level_width"]
    assert r.act_gen == fx["act_gen"] and r.act_dist == fx["act_dist"]
    assert r.outdeg_hist == fx["outdeg_hist"]
    # the same from Init (KC_DEFER_REDO=0)
    monkeypatch.setenv("KC_DEFER_REDO", "0")
    r0 = run(np=2, max_levels=40, keep_trace=False)
    assert r0.defer_fallback and r0.defer_redo_level == 1
    assert (r0.level_width, r0.act_gen, r0.act_dist) == (r.level_width, r.act_gen, r.act_dist)


@pytest.mark.parametrize("direct", ["1", "0"])
@pytest.mark.parametrize("key,kw", [("variant3", dict(variant=3)), ("variant2", dict(variant=2))])
def test_deferred_error_redone_exactly(fixtures, monkeypatch, key, kw, direct):
    # an error on a deferred wide level (Model_1 on the wide path).  An
    # Assert is found among the level's own parents: the run is redone on
    # the materialising path from that level.  An invariant violation among
    # the states the level rebuilt (the previous level's emit would have
    # found it) is reported directly — the lowest rebuilt index, counters and
    # ClaimSet put back as that emit left them (KC_DEFER_DIRECT=0: redone from
    # the previous level instead).  Trace state for state either way.
    monkeypatch.setenv("KC_DEFER_DIRECT", direct)
    fx = fixtures[key]
    with ModelChecker(ModelConfig(chunk_states=1 << 20, **kw)) as mc:
        r = mc.run()
    if key == "variant2" and direct == "1":
        assert r.error == "invariant" and not r.defer_fallback and r.defer_redo_level == 0
    else:
        assert r.defer_fallback
        assert r.defer_redo_level == fx["err_level"] - (1 if r.error == "invariant" else 0)
    assert (r.error_level, r.trace_len) == (fx["err_level"], fx["trace_len"])
    assert [list(map(int, t)) for t in r.trace] == fx["trace"]
    # every partial count as the exact (materialising) path reports it
    monkeypatch.setenv("KC_DEFER", "0")
    with ModelChecker(ModelConfig(chunk_states=1 << 20, **kw)) as mc:
        e = mc.run()
    assert not e.defer_fallback and e.deferred_states == 0
    for k in ("distinct", "generated", "depth", "level_width", "act_gen", "act_dist", "outdeg_hist", "error_level",
              "error_invariant", "trace_len", "complete", "queue_left"):
        assert getattr(r, k) == getattr(e, k), k
    assert [list(map(int, t)) for t in r.trace] == [list(map(int, t)) for t in e.trace]


def test_deferred_invariant_np2_lost_update(fixtures, monkeypatch):
    # NP=2's resourceVersion race (NoLostUpdate, depth 25) found among a
    # deferred level's rebuilt states: reported without a redo, everything
    # as the materialising path reports it
    fx = fixtures["np2_variant1_lost_update"]
    r = run(np=2, variant=1, invariants=7)
    assert r.error_invariant == "NoLostUpdate" and not r.defer_fallback
    assert (r.error_level, r.trace_len) == (fx["err_level"], fx["trace_len"])
    monkeypatch.setenv("KC_DEFER", "0")
    e = run(np=2, variant=1, invariants=7)
    for k in ("distinct", "generated", "depth", "level_width", "act_gen", "act_dist", "outdeg_hist", "error_level",
              "trace_len"):
        assert getattr(r, k) == getattr(e, k), k
    assert [list(map(int, t)) for t in r.trace] == [list(map(int, t)) for t in e.trace]


def test_deferred_trace_in_host_memory(fixtures):
    # trace_host: the trace lives in pinned host RAM, the links in HBM
    fx = fixtures["np2_40levels"]
    r = run(np=2, max_levels=40, trace_host=True)
    assert r.deferred_states > 0 and not r.defer_fallback
    assert r.level_width == fx["level_width"] and r.act_dist == fx["act_dist"]


@pytest.mark.parametrize("defer", ["1", "0"])
def test_wide_level_state_set_identical(oracle, monkeypatch, defer):
    # a captured WIDE level of the NP=2 model (level 30: 35,224 states, past
    # the narrow path): on the deferred frontier it is materialised for the
    # capture; same states in the same FIFO order as the oracle
    monkeypatch.setenv("KC_DEFER", defer)
    with ModelChecker(ModelConfig(np=2, max_levels=32)) as mc:
        mc.capture_level(30)
        mc.run()
        got = mc.level_tuples(30)
    want = oracle.level_tuples(oracle.config(np_=2), 30)
    assert got.shape == want.shape == (35224, got.shape[1])
    assert np.array_equal(got, want)


# --- first-claim mode (KC_FIRST_CLAIM=1, k_claim FIRST): the first inserter
# of a fingerprint wins, as in a multi-worker TLC run; no settle passes.
# Counts, generated per action, widths, error kinds, levels and trace lengths
# are the exact path's; which copy of a same-level duplicate wins is not
# deterministic, so per-action distinct counts only sum to the same total and
# a trace is checked as a real behaviour from an Init state.
def _valid_trace(oracle, cfg, trace):
    init = {tuple(map(int, t)) for t in oracle.level_tuples(cfg, 1)}
    assert tuple(trace[0]) in init
    for a, b in zip(trace, trace[1:]):
        succ, _ = oracle.successors(cfg, a)
        assert any(list(map(int, x)) == b for _, x in succ)


@pytest.mark.parametrize("env", [{}, {"KC_DEFER": "0"}, {"KC_DEFER_SLACK": "0.001"}, {"KC_CHUNK_SCAN": "0"}])
def test_first_claim_counts(model1, fixtures, monkeypatch, env):
    monkeypatch.setenv("KC_FIRST_CLAIM", "1")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    r = run(chunk_states=1 << 20)          # every level on the wide path
    assert (r.distinct, r.generated, r.depth) == (model1.distinct, model1.generated, model1.depth)
    assert r.level_width == model1.level_width and r.act_gen == model1.act_gen
    assert sum(r.act_dist.values()) == sum(model1.act_dist.values())
    assert r.complete and r.error is None
    assert r.claim_mode == "first"
    fx = fixtures["np2_40levels"]
    r = run(np=2, max_levels=40)
    assert r.level_width == fx["level_width"] and r.act_gen == fx["act_gen"]
    # (the mode is decided after the deferred frontier forces the tile scan
    # on, so KC_TSCAN=0 does not drop it: ADVICE r5)
    monkeypatch.setenv("KC_TSCAN", "0")
    r = run(chunk_states=1 << 20)
    assert r.claim_mode == ("minimum" if env.get("KC_DEFER") == "0" else "first")
    assert r.level_width == model1.level_width


@pytest.mark.parametrize("key,kw,kind", [("nc2", dict(nc=2), "assertion"), ("variant2", dict(variant=2), "invariant"),
                                         ("variant3", dict(variant=3), "assertion"),
                                         ("variant4", dict(variant=4), "invariant"),
                                         ("ns0", dict(ns=0), "deadlock")])
def test_first_claim_errors(fixtures, oracle, monkeypatch, key, kw, kind):
    monkeypatch.setenv("KC_FIRST_CLAIM", "1")
    fx = fixtures[key]
    r = run(chunk_states=1 << 20, **kw)
    assert r.error == kind
    assert (r.error_level, r.trace_len) == (fx.get("err_level", fx["trace_len"]), fx["trace_len"])
    cfg = oracle.config(nc=kw.get("nc", 1), ns=kw.get("ns", 1), variant=kw.get("variant", 0))
    _valid_trace(oracle, cfg, [list(map(int, t)) for t in r.trace])
    # found on a deferred level and reported there: an Assert or deadlock key
    # from the states k_claim rebuilt, an invariant violation among them as
    # the level before's (no redo of the whole run from Init)
    assert r.claim_mode == "first" and not r.defer_fallback, (r.defer_fallback, r.defer_redo_level)


# --- round 6: the compact ClaimSet of the first-claim mode (8-B fp-word
# slots, DevClaimSet::compact; KC_CLAIM_COMPACT=0 keeps 16-B slots): the same
# counts through the wide and narrow paths and the rehash growth (NP=2's 40
# levels grow the table from 2^20 slots), and the same fingerprint set
# (check_fps' minimum gap over every stored fingerprint equals the default
# mode's, whose table holds the same states)
def test_first_claim_compact(model1, fixtures, monkeypatch):
    with ModelChecker(ModelConfig()) as mc:
        mc.run()
        gap0, _ = mc.check_fps()
    fx = fixtures["np2_40levels"]
    for compact in ("1", "0"):
        monkeypatch.setenv("KC_CLAIM_COMPACT", compact)
        with ModelChecker(ModelConfig(first_claim=True)) as mc:
            r = mc.run()
            gap, _ = mc.check_fps()
            assert r.claim_mode == "first" and r.complete
            assert (r.distinct, r.generated, r.depth) == (model1.distinct, model1.generated, model1.depth)
            assert r.level_width == model1.level_width and gap == gap0
            r = mc.run()                      # the kept table, cleared (compact: half the bytes)
            assert r.level_width == model1.level_width
        r = run(np=2, max_levels=40, first_claim=True)
        assert r.level_width == fx["level_width"] and r.act_gen == fx["act_gen"]
        assert r.fpset_slots >= 1 << 21       # grown by rehash
