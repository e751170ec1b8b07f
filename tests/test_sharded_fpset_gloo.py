"""The sharded FPSet stress driver (kubecheck.sharded_fpset) over gloo with
world_size 1, 2 and 3 on CPU: every fingerprint lands on its owner rank, the
total size equals the number of distinct inserts, exactly half the lookups
are found, and the totals do not depend on the number of ranks.  Also pins
the library's stress stream (kc_stress_fp) to its definition."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, batch, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tla-kubernetes_amd"))
    import torch.distributed as dist
    from cpu_fpset_shard import CpuFPSetShard
    from kubecheck.sharded_fpset import ShardedFPSetStress

    dist.init_process_group("gloo", rank=rank, world_size=world)
    be = CpuFPSetShard(rank, world)
    r = ShardedFPSetStress(be).run(n, batch, n)
    r["misrouted"] = be.misrouted
    json.dump(r, open(os.path.join(outdir, f"r{rank}.json"), "w"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_stress_totals(tmp_path, world):
    n, batch = 6000, 1024          # several rounds, the last one ragged
    mp.spawn(_worker, args=(world, _free_port(), n, batch, str(tmp_path)), nprocs=world, join=True)
    outs = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    for o in outs:
        assert o["misrouted"] == 0
        assert (o["size"], o["inserted_new"], o["found"]) == (n, n, n // 2)
    assert sum(o["local_size"] for o in outs) == n
    if world > 1:
        assert outs[0]["fps_sent"] > 0


def test_stream_matches_library():
    import kubecheck
    from cpu_fpset_shard import stream

    seed, n = 0x5EED0000, 10_000_000_000
    idx = [0, 1, 2, 3, 1000, 12345, n - 1]
    for i in idx:
        assert kubecheck.stress_fp(seed, 0, n, i) == int(stream(seed, 0, n, i, 1)[0])
        assert kubecheck.stress_fp(seed, 1, n, i) == int(stream(seed, 1, n, i, 1)[0])
    # a bijection: distinct inputs, distinct normalised fingerprints
    fps = stream(seed, 0, n, 0, 200_000)
    assert len(set(fps.tolist())) == 200_000
    assert (fps < np.uint64(1 << 63)).all() and (fps != 0).all()


def test_key_map_orders_high_ranks():
    # error keys of ranks >= 8 are >= 2^63; the int64 collectives
    # must keep them ordered and below "no error"
    from kubecheck.distributed import NONE_KEY, i64_to_key, key_to_i64

    keys = [(r << 60) | (5 << 16) | 1 for r in range(15)] + [NONE_KEY]
    mapped = [key_to_i64(k) for k in keys]
    assert all(-(1 << 63) <= v < (1 << 63) for v in mapped)
    assert sorted(mapped) == mapped
    assert [i64_to_key(v) for v in mapped] == keys
    assert key_to_i64(NONE_KEY) == (1 << 63) - 1
