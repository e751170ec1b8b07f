"""The native sharded loop's all-to-all plan (kc_exchange_plan; the exchange
of SURVEY §8(e) step 4, issued to RCCL as grouped ncclSend/ncclRecv pieces
by RcclComm and replayed with device copies by the one-process emulation).

Host only: for world 1..9, random and skewed count matrices and piece sizes
down to 1 record, every rank's plan must pair with its peers' exactly as
RCCL pairs point-to-point calls (the k-th send from s to d with the k-th
receive at d from s, equal sizes), cover each send/receive buffer once in
rank order, and move every record to the right place (simulated)."""
import ctypes as C

import numpy as np
import pytest

from kubecheck import load


def plan(world, me, Mx, piece):
    lib = load()
    m = np.ascontiguousarray(Mx, dtype=np.uint64)
    n = lib.kc_exchange_plan(world, me, m.ctypes.data_as(C.POINTER(C.c_uint64)), piece, None, 0)
    assert n >= 0
    out = np.zeros(4 * max(n, 1), dtype=np.uint64)
    assert lib.kc_exchange_plan(world, me, m.ctypes.data_as(C.POINTER(C.c_uint64)), piece,
                                out.ctypes.data_as(C.POINTER(C.c_uint64)), n) == n
    return [tuple(int(v) for v in out[4 * k:4 * k + 4]) for k in range(n)]


def matrices():
    rng = np.random.default_rng(7)
    for world in range(1, 10):
        yield world, rng.integers(0, 40, size=(world, world))
        m = np.zeros((world, world), dtype=np.int64)
        m[0, :] = 97                      # one hot sender
        m[:, world - 1] += 13             # one hot receiver
        yield world, m
        yield world, np.zeros((world, world), dtype=np.int64)


@pytest.mark.parametrize("piece", [1, 3, 16, 1 << 20])
def test_exchange_plan_pairs_and_delivers(piece):
    for world, Mx in matrices():
        plans = [plan(world, r, Mx, piece) for r in range(world)]
        # send buffers: record value = (src, dst, j-th record for dst)
        send = []
        for s in range(world):
            buf = []
            for d in range(world):
                buf += [(s, d, j) for j in range(int(Mx[s, d]))]
            send.append(buf)
        recv = [[None] * int(Mx[:, d].sum()) for d in range(world)]
        for r, p in enumerate(plans):
            assert all(0 < n <= piece for _, _, _, n in p)
            # sends cover [0, sum of row) and receives [0, sum of column), in peer order
            soff = [o for _, snd, o, _ in p if snd]
            roff = [o for _, snd, o, _ in p if not snd]
            assert soff == sorted(soff) and roff == sorted(roff)
            assert sum(n for _, snd, _, n in p if snd) == int(Mx[r, :].sum())
            assert sum(n for _, snd, _, n in p if not snd) == int(Mx[:, r].sum())
        for s in range(world):
            for d in range(world):
                sends = [(o, n) for peer, snd, o, n in plans[s] if snd and peer == d]
                recvs = [(o, n) for peer, snd, o, n in plans[d] if not snd and peer == s]
                assert [n for _, n in sends] == [n for _, n in recvs]
                for (so, n), (ro, _) in zip(sends, recvs):
                    recv[d][ro:ro + n] = send[s][so:so + n]
        for d in range(world):
            want = []
            for s in range(world):
                want += [(s, d, j) for j in range(int(Mx[s, d]))]
            assert recv[d] == want


def test_exchange_plan_bad_args():
    lib = load()
    m = np.zeros(4, dtype=np.uint64)
    assert lib.kc_exchange_plan(2, 2, m.ctypes.data_as(C.POINTER(C.c_uint64)), 1, None, 0) == -22
    assert lib.kc_exchange_plan(0, 0, m.ctypes.data_as(C.POINTER(C.c_uint64)), 1, None, 0) == -22
