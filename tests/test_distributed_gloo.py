"""The sharded BFS driver (kubecheck.distributed) over the gloo backend with
world_size 2 and 3 on CPU: per-level widths, totals, per-action generated
counts and error traces must equal the single-process results (CPU oracle
fixtures) — totals do not depend on the number of ranks."""
import json
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kw, outdir, round_bytes=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tla-kubernetes_amd"))
    import torch.distributed as dist
    from cpu_shard import CpuShard
    from kubecheck import ModelConfig
    from kubecheck.distributed import ShardedModelChecker

    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = ModelConfig(**kw)
    mc = ShardedModelChecker(cfg, CpuShard(cfg, rank, world))
    if round_bytes:
        mc.A2A_ROUND_BYTES = round_bytes     # force the multi-round exchange
    res = mc.run()
    json.dump(res, open(os.path.join(outdir, f"r{rank}.json"), "w"))
    dist.destroy_process_group()


def run_sharded(tmp_path, world, round_bytes=None, **kw):
    mp.spawn(_worker, args=(world, _free_port(), kw, str(tmp_path), round_bytes), nprocs=world,
             join=True)
    outs = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    for o in outs:
        o.pop("seconds")
    for o in outs[1:]:
        assert o == outs[0]          # every rank agrees on the global result
    return outs[0]


@pytest.mark.parametrize("world,round_bytes", [(2, None), (3, None), (3, 4096)])
def test_sharded_counts_match_single(tmp_path, fixtures, world, round_bytes):
    # round_bytes=4096: the record exchange runs in many small all-to-all
    # rounds (the path large levels take; kubecheck.distributed._exchange)
    fx = fixtures["model1_fail0_timeout0"]
    r = run_sharded(tmp_path, world, round_bytes=round_bytes, can_fail=False, can_timeout=False)
    assert r["level_width"] == fx["level_width"]
    assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
    assert r["act_gen"] == fx["act_gen"]
    assert sum(r["act_dist"].values()) + r["init"] == r["distinct"]
    assert r["complete"] and r["error"] is None


def test_sharded_max_levels(tmp_path, fixtures):
    fx = fixtures["model1_fail0_timeout0"]
    r = run_sharded(tmp_path, 2, max_levels=20, can_fail=False, can_timeout=False)
    assert r["level_width"] == fx["level_width"][:20] and r["depth"] == 20
    assert not r["complete"] and r["error"] is None


def test_sharded_assertion_trace(tmp_path, fixtures, oracle):
    fx = fixtures["nc2"]
    r = run_sharded(tmp_path, 2, nc=2)
    assert r["error"] == "assertion" and r["error_action"] == "C4"
    assert r["error_level"] == 10 and r["trace_len"] == fx["trace_len"] == 10
    assert r["level_width"] == fx["level_width"]
    # the trace is a real behaviour: each state is a successor of the previous
    cfg = oracle.config(nc=2)
    for a, b in zip(r["trace"], r["trace"][1:]):
        succ, _ = oracle.successors(cfg, a)
        assert any(list(map(int, x)) == b for _, x in succ)
    _, fail = oracle.successors(cfg, r["trace"][-1])
    assert fail == "C4"


def test_sharded_invariant_trace(tmp_path, fixtures):
    fx = fixtures["variant2"]
    r = run_sharded(tmp_path, 2, variant=2)
    assert r["error"] == "invariant" and r["error_invariant"] == "OnlyOneVersion"
    assert r["trace_len"] == fx["trace_len"] and r["error_level"] == fx["err_level"]


def test_owner_function_matches_library():
    import kubecheck
    from kubecheck.distributed import owner

    lib = kubecheck.load()
    rng = __import__("numpy").random.default_rng(1)
    for fp in rng.integers(1, 2**63, size=2000, dtype="uint64"):
        for w in (2, 3, 8):
            assert owner(int(fp), w) == lib.kc_shard_owner(int(fp), w)


@pytest.mark.parametrize("key,kw,kind", [("variant5", dict(variant=5), "invariant"),
                                         ("ns0", dict(ns=0), "deadlock"),
                                         ("variant3", dict(variant=3), "assertion")])
def test_sharded_error_paths(tmp_path, fixtures, key, kw, kind):
    # variant5: an Init state violates OnlyOneVersion (the sharded Init-state
    # key 0x12); ns0: deadlock; variant3: C2's Assert
    fx = fixtures[key]
    r = run_sharded(tmp_path, 2, **kw)
    assert r["error"] == kind
    assert (r["error_level"], r["trace_len"]) == (fx["err_level"], fx["trace_len"])
    if kind == "assertion":
        assert r["error_action"] == fx["err_action"]
    assert r["trace"][0] == fx["trace"][0]


def test_bench_self_launch_two_ranks():
    # `python bench.py --gpus 2` with no launcher around it must start the two
    # ranks itself (torch.distributed.run as a child process, 127.0.0.1)
    import subprocess

    root = os.path.dirname(HERE)
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launcher-check"],
                         capture_output=True, text=True, timeout=300, cwd=root,
                         env={k: v for k, v in os.environ.items()
                              if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")})
    assert out.returncode == 0, out.stderr[-2000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
    rep = json.loads(line)
    assert rep["world"] == 2 and rep["n_gpus"] == 2 and rep["master_addr"] == "127.0.0.1"
    assert sorted(r[0] for r in rep["ranks"]) == [0, 1] and all(r[1] == 2 for r in rep["ranks"])
    assert sorted(r[2] for r in rep["ranks"]) == [0, 1]


@pytest.mark.parametrize("max_levels", [0, 1])
def test_sharded_init_violation_is_level1(tmp_path, fixtures, max_levels):
    # variant 5: an Init state violates OnlyOneVersion.  It is level 1's error
    # even when level 1 is not expanded (max_levels=1), and ahead of anything
    # level 1's expansion finds (it was min-merged with Assert
    # keys and lost at max_levels=1)
    r = run_sharded(tmp_path, 2, variant=5, max_levels=max_levels)
    assert r["error"] == "invariant" and r["error_level"] == 1
    assert r["trace_len"] == fixtures["variant5"]["trace_len"] == 1
