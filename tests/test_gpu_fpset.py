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
