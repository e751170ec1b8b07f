"""Host emulation of the kc_shard_* stage protocol (TEST INFRASTRUCTURE).

Lets the product's distributed driver (kubecheck.distributed) run under the
gloo backend on CPU: same record layout (packed state words, fingerprint,
key), same owner function, same key order — computed with the product's
host-compiled spec lowering (kc_spec_*), one state at a time."""
import numpy as np
import torch

import kubecheck
from kubecheck import ACTIONS, Spec
from kubecheck.distributed import NONE_KEY, owner

KEY_INIT = 0xF << 60


class CpuShard:
    device_type = "cpu"

    def __init__(self, cfg, rank, world):
        self.cfg, self.rank, self.world = cfg, rank, world
        self.spec = Spec(cfg)
        self.W = self.spec.state_words
        self.record_bytes = 8 * (self.W + 2)

    def init(self):
        self.seen, self.frontier, self.pkeys = set(), [], [[]]
        self.act_gen = [0] * len(ACTIONS)
        self.act_dist = [0] * len(ACTIONS)
        self.generated = 0
        self.init_err = NONE_KEY
        for k, t in enumerate(self.spec.init()):
            fp = self.spec.fingerprint(t)
            if owner(fp, self.world) != self.rank:
                continue
            self.seen.add(fp)
            self.frontier.append(t)
            self.pkeys[0].append(KEY_INIT | k)
            if self.spec.check_invariants(t) is not None:
                # (HipShard's key: the Init state's index in TLC's order, then the rank)
                self.init_err = min(self.init_err, (k << 16) | (self.rank << 8) | 0x12)
        self.n_init = len(self.frontier)
        self.init_key = self.init_err
        return len(self.frontier)

    def init_error(self):
        return self.init_key

    def expand(self):
        err, self.init_err = self.init_err, NONE_KEY
        init_violated = err != NONE_KEY            # then it is THE error (HipShard does the same)
        local, per_owner = set(), [[] for _ in range(self.world)]
        for i, s in enumerate(self.frontier):
            succ, fail = self.spec.successors(s)
            if succ is None:
                if not init_violated:
                    err = min(err, (self.rank << 60) | (i << 16) | 1)
                continue
            if not succ and self.cfg.check_deadlock and not init_violated:
                err = min(err, (self.rank << 60) | (i << 16) | 3)
            for t, (a, x) in enumerate(succ):
                self.act_gen[ACTIONS.index(a)] += 1
                self.generated += 1
                fp = self.spec.fingerprint(x)
                if fp in local:
                    continue
                local.add(fp)
                key = (self.rank << 60) | (i << 16) | (t << 8) | ACTIONS.index(a)
                per_owner[owner(fp, self.world)].append(
                    np.concatenate([self.spec.pack(x), np.array([fp, key], dtype=np.uint64)]))
        self.per_owner = per_owner
        return [len(p) for p in per_owner], err

    def pack(self, send):
        rows = [r for p in self.per_owner for r in p]
        if rows:
            arr = np.ascontiguousarray(np.stack(rows).astype(np.uint64)).view(np.int64).reshape(-1)
            send[: arr.size].copy_(torch.from_numpy(arr))      # int64 word buffer

    def insert(self, recv, n):
        err, batch, nxt, keys = NONE_KEY, set(), [], []
        if n:
            recs = recv[: n * (self.W + 2)].numpy().copy().view(np.uint64).reshape(n, self.W + 2)
            for r in recs:
                fp, key = int(r[self.W]), int(r[self.W + 1])
                if fp in batch:
                    continue
                batch.add(fp)
                if fp in self.seen:
                    continue
                self.seen.add(fp)
                t = self.spec.unpack(r[: self.W])
                nxt.append(t)
                keys.append(key)
                self.act_dist[key & 0xFF] += 1
                if self.spec.check_invariants(t) is not None:
                    err = min(err, (key & ~0xFF) | 2)
        self.next, self.next_keys = nxt, keys
        return len(nxt), err

    def advance(self):
        self.frontier = self.next
        self.pkeys.append(self.next_keys)

    def parent_key(self, level, idx):
        return self.pkeys[level - 1][idx]

    def result(self):
        return {"act_gen": self.act_gen, "act_dist": self.act_dist, "init": self.n_init,
                "generated": self.generated, "distinct": len(self.seen), "fpset_slots": 0}
