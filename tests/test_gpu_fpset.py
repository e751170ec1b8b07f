"""GPU FPSet (the tlc2.tool.fp.FPSet drop-in) against a Python set with TLC's
sequential put() semantics, plus the StateQueue FIFO."""
import numpy as np
import pytest

import kubecheck
from kubecheck import FPSet, StateQueue

pytestmark = pytest.mark.gpu
MASK = (1 << 63) - 1


def norm(fp):
    fp &= MASK
    return fp or 1


def sequential_put(model: set, fps):
    out = []
    for fp in fps:
        k = norm(int(fp))
        out.append(k in model)
        model.add(k)
    return np.array(out)


def test_put_matches_sequential_semantics():
    rng = np.random.default_rng(7)
    model = set()
    with FPSet(1 << 12) as s:
        for _ in range(6):
            base = rng.integers(0, 2**64, size=20000, dtype=np.uint64)
            batch = np.concatenate([base, base[:5000], rng.choice(base, 3000)])   # in-batch dups
            rng.shuffle(batch)
            assert np.array_equal(s.put_batch(batch), sequential_put(model, batch))
        assert s.size() == len(model)
        probe = rng.integers(0, 2**64, size=50000, dtype=np.uint64)
        want = np.array([norm(int(x)) in model for x in probe])
        assert np.array_equal(s.contains_batch(probe), want)


def test_lowest_index_wins_within_batch():
    with FPSet(64) as s:
        seen = s.put_batch(np.array([5, 9, 5, 5, 9, 11], dtype=np.uint64))
        assert seen.tolist() == [False, False, True, True, True, False]


def test_msb_and_zero_normalisation():
    with FPSet(64) as s:
        assert s.put(0x8000000000000005) is False
        assert s.put(5) is True                   # MSB ignored
        assert s.put(0) is False                  # 0 -> 1
        assert s.put(1) is True
        assert s.size() == 2


def test_growth_rehash_keeps_everything():
    rng = np.random.default_rng(3)
    fps = rng.integers(0, 2**64, size=300000, dtype=np.uint64)
    with FPSet(16) as s:
        for chunk in np.array_split(fps, 30):
            s.put_batch(chunk)
        assert s.capacity() >= s.size() * 4 // 3
        assert s.contains_batch(fps).all()
        assert s.size() == len({norm(int(x)) for x in fps})


def test_check_fps_min_gap():
    fps = np.array([10, 1000, 1003, 5000, 1 << 40], dtype=np.uint64)
    with FPSet(64) as s:
        s.put_batch(fps)
        p = s.checkFPs()
        assert s.min_gap == 3 and abs(p - 1 / 3) < 1e-12


def test_stress_small():
    with FPSet(1 << 20) as s:
        ti, tl, found = s.stress(seed=0x5EED0000, n=1 << 20, batch=1 << 18, n_lookup=1 << 20)
        assert s.size() == 1 << 20 and found == 1 << 19
        assert ti > 0 and tl > 0


def test_state_queue_fifo():
    q = StateQueue(4, 100)
    a = np.arange(4 * 70, dtype=np.uint64).reshape(70, 4)
    q.enqueue(a[:40])
    got = q.dequeue(25)
    q.enqueue(a[40:])
    got = np.concatenate([got, q.dequeue(100)])
    assert np.array_equal(got, a) and q.size() == 0
    q.close()


# ---------------------------------------------------------------------------
# BASELINE.json configs[3] at full size: 1e10 device-generated fingerprints
# (the perm63 stream: all distinct, so every count below is exact)
N_FULL = 10_000_000_000
SEED = 0x5EED0000


@pytest.mark.parametrize("load", [0.5, 0.75])
def test_stress_full_size(load):
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cpu_fpset_shard import stream

    # slots = 4/3 capacity -> final load `load`, with room for the window
    # below (a put past the 3/4 growth threshold would double the table)
    cap = int((N_FULL + 100_000) / load * 3 / 4)
    with FPSet(capacity=cap) as s:
        ti, tl, found = s.stress(SEED, N_FULL, 1 << 24, N_FULL)
        assert s.size() == N_FULL                # no in-stream duplicates by construction
        assert found == N_FULL // 2              # even lookups present, odd absent
        assert abs(s.size() / s.capacity() - load) < 0.01
        # exact sequential-put agreement on a sampled window: 3000 inserted fps,
        # 3000 never-inserted fps, 2000 repeats inside the batch
        rng = np.random.default_rng(11)
        idx = rng.integers(0, N_FULL, size=3000, dtype=np.uint64)
        present = np.concatenate([stream(SEED, 0, N_FULL, int(i), 1) for i in idx])
        absent = stream(SEED, 1, N_FULL, 2 * 10**9, 6000)[1::2]     # odd lookup entries: absent
        window = np.concatenate([present, absent, rng.choice(np.concatenate([present, absent]), 2000)])
        rng.shuffle(window)
        model = set(int(x) for x in present)      # exactly the window's inserted members
        want, seen_in_batch = [], set()
        for x in window.tolist():
            want.append(x in model or x in seen_in_batch)
            if x not in model:
                seen_in_batch.add(x)
        got = s.put_batch(window)
        assert np.array_equal(got, np.array(want))
        assert s.size() == N_FULL + len(set(absent.tolist()))
        assert ti > 0 and tl > 0


def test_single_put_from_many_threads():
    # TLC workers call put(long) concurrently: flat-combined batches must give
    # every fingerprint exactly one "new" answer across all threads
    import threading

    rng = np.random.default_rng(5)
    pool = rng.integers(1, 2**63, size=4000, dtype=np.uint64).tolist()
    results = [[] for _ in range(8)]
    with FPSet(1 << 16) as s:
        def worker(k):
            r = np.random.default_rng(100 + k)
            for fp in r.choice(pool, 1500).tolist():
                results[k].append((fp, s.put(fp)))
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        new = {}
        for res in results:
            for fp, seen in res:
                if not seen:
                    new[fp] = new.get(fp, 0) + 1
        touched = {fp for res in results for fp, _ in res}
        assert set(new) == touched and all(v == 1 for v in new.values())
        assert s.size() == len(touched)
        assert all(s.contains(fp) for fp in list(touched)[:200])
        assert 0 < s.combine_rounds() <= 8 * 1500 + 200


@pytest.mark.parametrize("world", [1, 3, 8])
def test_partition_dev_stable(world):
    import torch
    rng = np.random.default_rng(world)
    a = rng.integers(0, 2**64, size=100_003, dtype=np.uint64)
    with FPSet(1 << 10) as s:
        src = torch.from_numpy(a.view(np.int64)).cuda()
        out = torch.empty_like(src)
        counts = s.partition_dev(src, a.size, world, out)
        got = out.cpu().numpy().view(np.uint64)
    own = np.array([(((int(x) & MASK) or 1) * world) >> 63 for x in a])
    assert counts == [int((own == r).sum()) for r in range(world)]
    assert np.array_equal(got, a[np.argsort(own, kind="stable")])


def test_sharded_routing_emulated():
    # R ranks' tables on one GPU: partition each rank's share, route every
    # owner slice to its table, then the tables are disjoint and complete
    import torch
    from kubecheck import stress_fps_dev
    R, n = 4, 1 << 22
    tables = [FPSet(1 << 21) for _ in range(R)]
    gen = torch.empty(n // R, dtype=torch.int64, device="cuda")
    part = torch.empty_like(gen)
    for r in range(R):
        stress_fps_dev(SEED, 0, n, r * (n // R), n // R, gen)
        counts = tables[r].partition_dev(gen, n // R, R, part)
        off = 0
        for o in range(R):
            if counts[o]:
                assert tables[o].insert_count_dev(part[off:off + counts[o]], counts[o]) == counts[o]
            off += counts[o]
    assert sum(t.size() for t in tables) == n
    probe = torch.empty(n, dtype=torch.int64, device="cuda")
    stress_fps_dev(SEED, 0, n, 0, n, probe)
    assert sum(t.contains_count_dev(probe, n) for t in tables) == n     # each fp in exactly one table
    for t in tables:
        t.close()
