"""Seen-set spill (kc_model_config.seen_hbm_bytes): the engine's seen-set
under an HBM budget, TLC's OffHeapDiskFPSet role (MC.out:5: an in-memory
table flushed into sorted runs that later lookups also check).

The hot ClaimSet is flushed into sorted runs in pinned host RAM and, past
seen_host_bytes, in spill files; every chunk's new fingerprints are checked
against the runs on the GPU.  Results must be identical to the unbounded
seen-set's and to the golden counts:

* Model_1 equals MC.out (totals, depth, widths, per-action counts) through
  the host tier, the file tier (small staging windows: many windows, most
  skipped), with the Bloom filters off (every query reads the runs), and
  with every host run read by the streaming merge-probe;
* every error kind, with its trace, state for state against the in-HBM run;
* the NP=2 model's first 55 levels through the file tier;
* the full NP=2 model (740,607,995 states) with its seen-set capped at 4 GiB
  of HBM (natural size 32 GiB), exact against tests/golden/np2_full.json."""
import os

import pytest

from kubecheck import KubecheckError, ModelChecker, ModelConfig

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _run(**kw):
    with ModelChecker(ModelConfig(**kw)) as mc:
        r = mc.run()
        gap = mc.check_fps() if kw.get("check_fps_too") else None
    return r, gap


def _same(a, b):
    assert (a.distinct, a.generated, a.depth, a.queue_left, a.complete) == (
        b.distinct, b.generated, b.depth, b.queue_left, b.complete)
    assert a.level_width == b.level_width
    assert a.act_gen == b.act_gen and a.act_dist == b.act_dist
    assert a.outdeg_hist == b.outdeg_hist
    assert (a.error, a.error_action, a.error_invariant, a.error_level, a.trace_len) == (
        b.error, b.error_action, b.error_invariant, b.error_level, b.trace_len)
    assert [list(map(int, t)) for t in a.trace] == [list(map(int, t)) for t in b.trace]


@pytest.fixture(scope="module")
def model1_ref():
    with ModelChecker(ModelConfig()) as mc:
        r = mc.run()
        gap = mc.check_fps()
    return r, gap


@pytest.mark.parametrize("tier", ["host", "disk", "no_filter", "host_budget_no_dir", "merge_probe"])
def test_seen_spill_model1(model1_ref, mcout, fixtures, tmp_path, monkeypatch, tier):
    ref, ref_gap = model1_ref
    kw = dict(seen_hbm_bytes=4 * MiB)
    if tier == "disk":
        kw.update(seen_host_bytes=256 << 10, spill_dir=str(tmp_path))
        monkeypatch.setenv("KC_COLD_WINDOW", "4096")
    if tier == "no_filter":
        monkeypatch.setenv("KC_COLD_BLOOM_BITS", "0")
    if tier == "merge_probe":   # every host run probed by the streaming merge (coldset.hip), none cached in HBM
        monkeypatch.setenv("KC_COLD_MERGE_DIV", "100000000")
        monkeypatch.setenv("KC_COLD_CACHE", "0")
    if tier == "host_budget_no_dir":
        kw.update(seen_host_bytes=256 << 10)
        with pytest.raises(KubecheckError) as e:
            _run(**kw)
        assert e.value.code == -12 and "no spill directory" in str(e.value)
        return
    with ModelChecker(ModelConfig(**kw)) as mc:
        r = mc.run()
        gap = mc.check_fps()
    _same(r, ref)
    assert (r.distinct, r.generated, r.depth) == (mcout["distinct"], mcout["generated"], mcout["depth"])
    assert r.level_width == fixtures["model1"]["level_width"]
    s = r.seen
    assert s["flushes"] >= 2 and s["cold_hits"] > 0 and s["cold_queries"] >= r.distinct
    assert s["peak_hbm_bytes"] <= 4 * MiB
    # every distinct state's fingerprint is in exactly one tier: checkFPs sees them all
    assert gap == ref_gap
    if tier == "disk":
        assert s["disk_bytes"] > 0
        assert os.listdir(tmp_path) == []       # spill files removed with the engine
    if tier in ("no_filter", "merge_probe"):
        assert s["filter_tests"] == 0          # (the streaming merge reads whole runs, no filters)
    else:
        assert 0 < s["filter_passed"] < s["filter_tests"]


@pytest.mark.parametrize("kw", [dict(nc=2), dict(variant=2), dict(variant=3), dict(variant=4),
                                dict(variant=5), dict(ns=0)])
def test_seen_spill_error_paths(kw):
    ref, _ = _run(**kw)
    r, _ = _run(**kw, seen_hbm_bytes=4 * MiB)
    assert r.error is not None
    _same(r, ref)


def test_seen_spill_np2_prefix_disk(fixtures, tmp_path, monkeypatch):
    # 55 levels, 23M states: a 2^24-slot hot table, runs past 64 MiB of host
    # RAM in files, 8 MiB staging windows
    monkeypatch.setenv("KC_COLD_WINDOW", str(1 << 20))
    fx = fixtures["np2_full"]
    r, _ = _run(np=2, max_levels=55, keep_trace=False, seen_hbm_bytes=512 * MiB, seen_host_bytes=64 * MiB,
                spill_dir=str(tmp_path), verbose=1)
    ref, _ = _run(np=2, max_levels=55, keep_trace=False)
    _same(r, ref)
    assert r.level_width == fx["level_width"][:55]
    s = r.seen
    assert s["disk_bytes"] > 0 and s["flushes"] >= 2 and s["peak_hbm_bytes"] <= 512 * MiB
    assert os.listdir(tmp_path) == []


def test_seen_spill_np2_full(fixtures):
    # the whole enlarged model with the seen-set capped at 4 GiB of HBM (its
    # natural size is a 2^31-slot, 32 GiB ClaimSet): older fingerprints in
    # sorted runs in pinned host RAM
    fx = fixtures["np2_full"]
    r, _ = _run(np=2, keep_trace=False, seen_hbm_bytes=4 << 30, verbose=1)   # (a line per level)
    assert (r.distinct, r.generated, r.depth) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r.level_width == fx["level_width"]
    assert r.act_gen == fx["act_gen"] and r.act_dist == fx["act_dist"]
    s = r.seen
    assert r.complete and s["flushes"] > 5 and s["peak_hbm_bytes"] <= 4 << 30
    assert s["cold_fps"] + 0 <= r.distinct
    print(f"\nNP=2 seen-set 4 GiB: {r.seconds:.2f} s, {s}")


@pytest.mark.parametrize("kw", [{}, dict(variant=3), dict(nc=2), dict(variant=1, invariants=7)])
def test_seen_spill_with_frontier_spill(model1_ref, fixtures, tmp_path, kw):
    # both spills at once (TLC's DiskStateQueue + OffHeapDiskFPSet, MC.out:5):
    # frontiers in a StateQueue over HBM/host/disk and the seen-set under a
    # 4 MiB budget; results equal the all-in-HBM engine's
    ref = model1_ref[0] if not kw else _run(**kw)[0]
    r, _ = _run(**kw, seen_hbm_bytes=4 * MiB, frontier_hbm_bytes=48 << 10, frontier_host_bytes=64 << 10,
                frontier_segment_states=384, spill_dir=str(tmp_path))
    _same(r, ref)
    if not kw:
        assert r.seen["flushes"] >= 2 and r.frontier_spilled_bytes > 0
    assert os.listdir(tmp_path) == []
