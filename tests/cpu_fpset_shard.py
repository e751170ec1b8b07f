"""Host emulation of the sharded-FPSet stages (TEST INFRASTRUCTURE).

Lets kubecheck.sharded_fpset.ShardedFPSetStress run under gloo on CPU: the
same stress stream (perm63, re-derived here in numpy from its definition in
include/kubecheck.h), the same owner function and a stable partition, with
a Python set as this rank's table."""
import numpy as np

M63 = np.uint64((1 << 63) - 1)


def perm63(x: np.ndarray) -> np.ndarray:
    """The stress stream's bijection of [0, 2^63) (xor-shifts and odd
    multiplies mod 2^63), uint64 numpy arithmetic wraps mod 2^64."""
    x = x.astype(np.uint64) & M63
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(31); x = (x * np.uint64(0x9e3779b97f4a7c15)) & M63
        x ^= x >> np.uint64(29); x = (x * np.uint64(0xbf58476d1ce4e5b9)) & M63
        x ^= x >> np.uint64(32); x = (x * np.uint64(0x94d049bb133111eb)) & M63
    return x ^ (x >> np.uint64(30))


def splitmix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9e3779b97f4a7c15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


def stream(seed: int, kind: int, n_ins: int, start: int, n: int) -> np.ndarray:
    i = np.arange(start, start + n, dtype=np.uint64)
    if kind == 0:
        return perm63(np.uint64(seed) + i)
    odd = (i & np.uint64(1)).astype(bool)
    x = np.where(odd, np.uint64(seed + n_ins) + i, np.uint64(seed) + splitmix64(i) % np.uint64(n_ins))
    return perm63(x)


def owners(fps: np.ndarray, world: int) -> np.ndarray:
    """floor(fp * R / 2^63) of normalised fps (exact, via Python ints)."""
    return np.array([((int(f) & ((1 << 63) - 1)) * world) >> 63 for f in fps], dtype=np.int64)


class CpuFPSetShard:
    device_type = "cpu"

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world
        self.table = set()
        self.misrouted = 0

    @staticmethod
    def _np(t, n):
        return t[:n].numpy().view(np.uint64)

    def gen(self, seed, kind, n_ins, start, n, out, stream_=None):
        if n:
            self._np(out, n)[:] = stream(seed, kind, n_ins, start, n)

    def partition(self, fps, n, world, out, stream_=None):
        a = self._np(fps, n).copy()
        o = owners(a, world)
        order = np.argsort(o, kind="stable")
        self._np(out, n)[:] = a[order]
        return [int((o == r).sum()) for r in range(world)]

    def insert(self, fps, n, stream_=None):
        a = self._np(fps, n)
        self.misrouted += int((owners(a, self.world) != self.rank).sum())
        before = len(self.table)
        self.table.update(int(x) for x in a)
        return len(self.table) - before

    def lookup(self, fps, n, stream_=None):
        return sum(int(x) in self.table for x in self._np(fps, n))

    def size(self):
        return len(self.table)
