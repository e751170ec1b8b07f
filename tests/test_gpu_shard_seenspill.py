"""The seen-set spill in the sharded loop (kc_model_config.seen_hbm_bytes per
rank): every rank's share of the fingerprints in a fixed hot ClaimSet,
flushed into sorted cold runs (pinned host RAM, then spill files) that each
level's winners are checked against on the GPU (shard.hip spill_check).  The
role of TLC's OffHeapDiskFPSet (MC.out:5) on every rank of the distributed
check the sharding replaces (KubeAPI___Model_1.launch:4-7).

Results must equal the unbounded sharded run's and the golden fixtures:
Model_1 at 2 and 4 emulated ranks through the host and file tiers, every
error kind with its trace, and the whole NP=2 model at 4 emulated ranks with
1 GiB of seen-set HBM per rank (tests/golden/np2_full.json).  The one-shard-
per-process case (HostComm at world 2) is in tests/test_gpu_hostcomm.py."""
import os

import pytest

from kubecheck import ModelConfig
from kubecheck.distributed import NativeShardedChecker

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def native(R, **kw):
    mc = NativeShardedChecker(ModelConfig(**kw), emulate=R)
    try:
        return mc.run()
    finally:
        mc.close()


def _same(a, b):
    for k in ("distinct", "generated", "depth", "level_width", "act_gen", "act_dist", "complete", "error"):
        assert a[k] == b[k], k
    for k in ("error_level", "trace_len", "trace", "error_action", "error_invariant"):
        assert a.get(k) == b.get(k), k


@pytest.mark.parametrize("R,budget,tier", [(2, 4 * MiB, "host"), (4, 3 * MiB, "host"), (2, 4 * MiB, "disk"),
                                           (2, 4 * MiB, "windows"), (3, 3 * MiB, "merge_probe")])
def test_shard_seen_spill_model1(fixtures, mcout, tmp_path, monkeypatch, R, budget, tier):
    ref = native(R)
    kw = dict(seen_hbm_bytes=budget)
    if tier == "disk":
        kw.update(seen_host_bytes=128 << 10, spill_dir=str(tmp_path))
        monkeypatch.setenv("KC_COLD_WINDOW", "4096")
    if tier == "windows":       # each level's cold check in windows of 256 queries (last to first)
        monkeypatch.setenv("KC_SEEN_QMAX", "256")
    if tier == "merge_probe":   # every host run probed by the streaming merge, none cached in HBM
        monkeypatch.setenv("KC_COLD_MERGE_DIV", "100000000")
        monkeypatch.setenv("KC_COLD_CACHE", "0")
    r = native(R, **kw)
    _same(r, ref)
    fx = fixtures["model1"]
    assert (r["distinct"], r["generated"], r["depth"]) == (mcout["distinct"], mcout["generated"], mcout["depth"])
    assert r["level_width"] == fx["level_width"]
    # the runs took part: flushes on every rank, and states found there
    assert r["seen_flushes"] >= R and r["seen_cold_hits"] > 0
    assert r["seen_cold_queries"] >= r["distinct"] - r["init"]
    assert r["narrow_levels"] == 0            # (the counted path at every level)
    if tier == "disk":
        assert os.listdir(tmp_path) == []     # spill files removed with the shards


@pytest.mark.parametrize("kw", [dict(nc=2), dict(variant=2), dict(variant=3), dict(variant=5), dict(ns=0),
                                dict(variant=1, invariants=7)])
def test_shard_seen_spill_errors(kw):
    ref = native(2, **kw)
    r = native(2, **kw, seen_hbm_bytes=4 * MiB)
    assert r["error"] is not None
    _same(r, ref)


def test_shard_seen_spill_budget_too_small():
    from kubecheck import KubecheckError
    with pytest.raises(KubecheckError) as e:
        native(2, seen_hbm_bytes=1 * MiB)
    assert "too small" in str(e.value)


def test_shard_seen_spill_np2_full_r4(fixtures):
    # the whole enlarged model on 4 emulated ranks, each rank's seen-set
    # capped at 1 GiB of HBM (a 2^25-slot hot table; its unbounded shard
    # grows to 2^29 slots): exact against the golden
    fx = fixtures["np2_full"]
    r = native(4, np=2, keep_trace=False, seen_hbm_bytes=1 << 30)
    assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r["level_width"] == fx["level_width"]
    assert r["complete"] and r["error"] is None
    assert r["seen_flushes"] > 4 and r["seen_cold_hits"] > 0
    print(f"\nNP=2 sharded R=4, seen-set 1 GiB per rank: {r['seconds']:.2f} s, flushes {r['seen_flushes']}, "
          f"cold fps {r['seen_cold_fps']}, queries {r['seen_cold_queries']}, hits {r['seen_cold_hits']}")


@pytest.mark.parametrize("R", [1, 2])
def test_shard_seen_spill_np2_lost_update(fixtures, R):
    # NP=2's resourceVersion race (variant 1, NoLostUpdate; BASELINE config
    # 5; 39,729 states to its depth 25) under a 3 MiB seen-set per rank (a
    # 2^16-slot hot table): the error, its level and its trace are the
    # unbounded sharded run's and the oracle's
    kw = dict(np=2, variant=1, invariants=7)
    ref = native(R, **kw)
    r = native(R, **kw, seen_hbm_bytes=3 * MiB)
    fx = fixtures["np2_variant1_lost_update"]
    assert r["error"] == "invariant" and r["error_invariant"] == "NoLostUpdate"
    assert (r["error_level"], r["trace_len"]) == (fx["err_level"], fx["trace_len"])
    _same(r, ref)
    if R == 1:
        assert r["seen_flushes"] >= 1


def test_shard_seen_spill_np2_prefix(fixtures):
    # NP=2's first 40 levels (1.7M states) at 2 ranks under 16 MiB each:
    # several flushes per rank and cold checks in several windows a level
    # (per-action distinct counts follow the ranks' claim order, not the
    # oracle's FIFO order: compared with the unbounded run at 2 ranks)
    fx = fixtures["np2_40levels"]
    r = native(2, np=2, max_levels=40, keep_trace=False, seen_hbm_bytes=16 * MiB)
    ref = native(2, np=2, max_levels=40, keep_trace=False)
    assert r["level_width"] == fx["level_width"]
    assert r["act_gen"] == fx["act_gen"] and r["act_dist"] == ref["act_dist"]
    assert r["seen_flushes"] >= 4 and r["seen_cold_hits"] > 0
