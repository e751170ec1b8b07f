"""The StateQueue plugin (kc_squeue_*; TLC's StateQueue seam, the recorded
run's DiskStateQueue, MC.out:5) and the engine's frontier spill.

* FIFO order through every tier (HBM, pinned host RAM, spill files) under
  random interleavings of host/device enqueues and dequeues, against a
  Python model of the queue;
* in-place device runs: reserve/commit written by a kernel, front/pop read
  in place;
* the budgets are honoured and exhausting them without a spill directory
  fails loudly;
* the engine with its frontiers in the queue (tiny HBM budgets: levels
  spill to host RAM and disk) gives results identical to the in-HBM engine
  and the oracle: totals, widths, per-action counts, outdegree, state sets,
  error traces; and the full NP=2 model against its golden counts."""
import os

import numpy as np
import pytest

import kubecheck
from kubecheck import KubecheckError, ModelChecker, ModelConfig, StateQueue

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    return torch


def _dev(a: np.ndarray):
    return _torch().from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


def test_fifo_through_all_tiers(tmp_path):
    torch = _torch()
    W, SEG = 6, 1000
    seg_b = SEG * W * 8
    q = StateQueue(W, device=0, segment_states=SEG, hbm_bytes=3 * seg_b, host_bytes=4 * seg_b,
                   spill_dir=str(tmp_path))
    rng = np.random.default_rng(7)
    model = []          # expected FIFO contents, row blocks
    nxt = 0
    peak_size = 0
    for step in range(300):
        op = rng.integers(0, 5)
        if op <= 1 or sum(len(b) for b in model) < 500:
            n = int(rng.integers(1, 2500))
            a = (np.arange(nxt, nxt + n, dtype=np.uint64)[:, None] * np.uint64(W)
                 + np.arange(W, dtype=np.uint64)[None, :]) ^ np.uint64(0x5A5A5A5A5A5A5A5A)
            nxt += n
            if op == 0:
                q.enqueue(a)
            else:
                q.enqueue_dev(_dev(a))
            model.append(a)
        else:
            n = int(rng.integers(1, 3000))
            want = np.concatenate(model)[:n] if model else np.zeros((0, W), np.uint64)
            if op == 2:
                got = q.dequeue(n)
            elif op == 3:
                out = torch.zeros((n, W), dtype=torch.int64, device="cuda")
                k = q.dequeue_dev(out, n)
                torch.cuda.synchronize()
                got = out[:k].cpu().numpy().view(np.uint64)
            else:           # peek at a random window, then pop
                size = q.size()
                off = int(rng.integers(0, max(size, 1)))
                m = min(n, size - off)
                if m > 0:
                    assert np.array_equal(q.peek(off, m), np.concatenate(model)[off:off + m])
                got = q.dequeue(n)
            assert np.array_equal(got, want[: len(got)]) and len(got) == len(want)
            rest = np.concatenate(model)[len(got):] if model else np.zeros((0, W), np.uint64)
            model = [rest] if len(rest) else []
        peak_size = max(peak_size, q.size())
        assert q.size() == sum(len(b) for b in model)
        st = q.stats()
        # the budget holds except for the segments being read and written
        assert st["hbm_bytes"] <= 4 * seg_b
    st = q.stats()
    assert st["spilled_host_bytes"] > 0 and st["spilled_disk_bytes"] > 0 and st["reloaded_bytes"] > 0
    assert peak_size > 7 * SEG
    rest = q.dequeue(q.size())
    assert np.array_equal(rest, np.concatenate(model) if model else np.zeros((0, W), np.uint64))
    assert q.size() == 0
    q.close()
    assert os.listdir(tmp_path) == []          # spill files are removed when read back


def test_in_place_reserve_commit_front_pop(tmp_path):
    # a kernel (the library's stress-stream generator) writes straight into
    # reserved tail runs; front() hands out head runs in place
    torch = _torch()
    SEED, N_INS = 0x5EED0000, 1 << 40
    q = StateQueue(1, device=0, segment_states=1 << 16, hbm_bytes=3 << 19, host_bytes=2 << 19,
                   spill_dir=str(tmp_path))
    written = 0
    lib = kubecheck.load()
    import ctypes as C
    for n in [1000, 65536, 70000, 5, 200000, 12345, 131072]:
        p = q.reserve_dev(n)
        assert lib.kc_stress_fps_dev(SEED, 0, N_INS, written, n, C.c_void_p(p), None) == 0
        q.commit(n)
        written += n
    torch.cuda.synchronize()
    assert q.size() == written
    assert q.stats()["spilled_host_bytes"] > 0
    want = torch.empty(written, dtype=torch.int64, device="cuda")
    kubecheck.stress_fps_dev(SEED, 0, N_INS, 0, written, want)
    off = 0
    while q.size():
        p, m = q.front_dev(0, 50000)
        assert 0 < m <= 50000
        got = torch.empty(m, dtype=torch.int64, device="cuda")
        q2 = StateQueue(1, 1 << 16, device=0)   # copy the run out through another queue's device path
        q2.enqueue_dev(p, m)
        assert q2.dequeue_dev(got, m) == m
        q2.close()
        torch.cuda.synchronize()
        assert torch.equal(got, want[off:off + m])
        q.pop(m)
        off += m
    assert off == written
    q.close()


def test_spill_at_scale(tmp_path):
    # 2^26 states (512 MiB) through a 128 MiB HBM and 128 MiB host budget
    torch = _torch()
    import ctypes as C
    SEED, N_INS = 0x5EED0000, 1 << 40
    n_tot, seg = 1 << 26, 1 << 22
    q = StateQueue(1, device=0, segment_states=seg, hbm_bytes=128 << 20, host_bytes=128 << 20,
                   spill_dir=str(tmp_path))
    lib = kubecheck.load()
    for start in range(0, n_tot, seg):
        p = q.reserve_dev(seg)
        assert lib.kc_stress_fps_dev(SEED, 0, N_INS, start, seg, C.c_void_p(p), None) == 0
        q.commit(seg)
    st = q.stats()
    assert st["seg_disk"] > 0 and st["seg_host"] > 0 and st["hbm_bytes"] <= 160 << 20
    out = torch.empty(seg, dtype=torch.int64, device="cuda")
    want = torch.empty(seg, dtype=torch.int64, device="cuda")
    for start in range(0, n_tot, seg):
        assert q.dequeue_dev(out, seg) == seg
        kubecheck.stress_fps_dev(SEED, 0, N_INS, start, seg, want)
        torch.cuda.synchronize()
        assert torch.equal(out, want)
    assert q.size() == 0 and q.stats()["reloaded_bytes"] >= n_tot * 8 - (128 << 20)
    q.close()


def test_budget_exhausted_fails_loudly():
    W, SEG = 4, 1024
    q = StateQueue(W, device=0, segment_states=SEG, hbm_bytes=2 * SEG * W * 8, host_bytes=SEG * W * 8)
    with pytest.raises(KubecheckError) as e:
        for _ in range(10):
            q.enqueue(np.zeros((SEG, W), dtype=np.uint64))
    assert e.value.code == -12 and "no spill directory" in str(e.value)
    q.close()


# ----------------------------------------------------------- engine spill
def _run(capture=0, **kw):
    with ModelChecker(ModelConfig(**kw)) as mc:
        if capture:
            mc.capture_level(capture)
        r = mc.run()
        lv = mc.level_tuples(capture) if capture else None
    return r, lv


def _same(a, b):
    assert (a.distinct, a.generated, a.depth, a.queue_left, a.complete) == (
        b.distinct, b.generated, b.depth, b.queue_left, b.complete)
    assert a.level_width == b.level_width
    assert a.act_gen == b.act_gen and a.act_dist == b.act_dist
    assert a.outdeg_hist == b.outdeg_hist
    assert (a.error, a.error_action, a.error_invariant, a.error_level, a.trace_len) == (
        b.error, b.error_action, b.error_invariant, b.error_level, b.trace_len)
    assert [list(map(int, t)) for t in a.trace] == [list(map(int, t)) for t in b.trace]


@pytest.mark.parametrize("budget", [
    dict(frontier_hbm_bytes=64 << 10, frontier_segment_states=512),                      # host RAM tier
    dict(frontier_hbm_bytes=48 << 10, frontier_host_bytes=64 << 10, frontier_segment_states=384,
         spill=True),                                                                      # + disk tier
    dict(frontier_hbm_bytes=1 << 30, trace_host=True),                                     # no spill, trace in RAM
])
def test_engine_spill_model1(fixtures, mcout, tmp_path, budget):
    b = dict(budget)
    if b.pop("spill", False):
        b["spill_dir"] = str(tmp_path)
    ref, ref_lv = _run(capture=51)
    r, lv = _run(capture=51, **b)
    _same(r, ref)
    assert np.array_equal(lv, ref_lv)
    assert (r.distinct, r.generated, r.depth) == (mcout["distinct"], mcout["generated"], mcout["depth"])
    assert r.level_width == fixtures["model1"]["level_width"]
    if b["frontier_hbm_bytes"] < (1 << 20):
        assert r.frontier_spilled_bytes > 0 and r.frontier_reloaded_bytes > 0
    assert os.listdir(tmp_path) == []


@pytest.mark.parametrize("kw", [dict(nc=2), dict(variant=2), dict(variant=3), dict(variant=4),
                                dict(variant=5), dict(ns=0)])
@pytest.mark.parametrize("mode", ["trace", "trace_host", "no_trace"])
def test_engine_spill_error_paths(kw, mode):
    # every error kind, with the trace file in HBM, in host RAM, or absent
    # (the failing parent then comes from the queue itself)
    extra = dict(keep_trace=mode != "no_trace", trace_host=mode == "trace_host")
    ref, _ = _run(**kw, keep_trace=mode != "no_trace")
    r, _ = _run(**kw, **extra, frontier_hbm_bytes=32 << 10, frontier_segment_states=256)
    assert r.error is not None
    assert (r.error, r.error_action, r.error_invariant, r.error_level, r.trace_len) == (
        ref.error, ref.error_action, ref.error_invariant, ref.error_level, ref.trace_len)
    assert [list(map(int, t)) for t in r.trace] == [list(map(int, t)) for t in ref.trace]
    assert r.level_width == ref.level_width


def test_engine_spill_np2_prefix(fixtures):
    fx = fixtures["np2_40levels"]
    r, _ = _run(np=2, max_levels=40, frontier_hbm_bytes=8 << 20, frontier_segment_states=1 << 15)
    assert r.level_width == fx["level_width"]
    assert r.act_gen == fx["act_gen"] and r.act_dist == fx["act_dist"]
    assert r.frontier_spilled_bytes > 0


def test_engine_spill_np2_full(fixtures):
    # the whole enlarged model with its frontiers capped at 512 MiB of HBM:
    # the 16M-state levels (768 MB) spill to host RAM and come back
    fx = fixtures["np2_full"]
    r, _ = _run(np=2, keep_trace=False, frontier_hbm_bytes=512 << 20)
    assert (r.distinct, r.generated, r.depth) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r.level_width == fx["level_width"]
    assert r.act_gen == fx["act_gen"] and r.act_dist == fx["act_dist"]
    assert r.complete and r.frontier_spilled_bytes > 0
    # (in-HBM, the two frontier buffers are sized by the successor count: GBs)
    assert r.frontier_peak_hbm_bytes < (3 << 29)


def test_legacy_capacity_is_a_bound():
    # kc_squeue_create(state_words, capacity_states, ...): the round-1
    # constructor's capacity stays a hard bound: enqueues past it
    # fail with -ENOMEM instead of growing the queue silently
    W = 4
    q = StateQueue(W, capacity=1024, device=0)
    q.enqueue(np.arange(1000 * W, dtype=np.uint64).reshape(-1, W))
    with pytest.raises(KubecheckError) as e:
        q.enqueue(np.zeros((25, W), dtype=np.uint64))
    assert e.value.code == -12 and "StateQueue full" in str(e.value)
    q.enqueue(np.zeros((24, W), dtype=np.uint64))           # exactly to capacity
    assert q.size() == 1024
    q.close()
