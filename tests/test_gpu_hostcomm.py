"""The native sharded level loop with ONE SHARD PER PROCESS at world 2 and 3,
on the one-GPU box: the layout `bench.py --gpus N` runs on N GPUs (RcclComm),
which RCCL itself refuses on one device ("duplicate GPU"; round-3 tools/gpu_r03_rccl2.sh, git history).
Here the collectives go over gloo through kc_group_create_host (HostComm,
shard_driver.hip): the same Group::run with one local shard and R > 1, the
device all-gather rows written by k_owner_totals, the exchange plan handed
over whole, the cross-rank broadcast of the error walk and the failure word.
Results must equal the fixtures exactly, as for the emulated ranks
(tests/test_gpu_shard.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    {"name": "model1", "kw": {}},
    {"name": "model1_hostrows", "kw": {}, "env": {"KC_DEVROW": "0"}},
    {"name": "model1_pieces", "kw": {}, "env": {"KC_PIECE_BYTES": "4096"}},
    {"name": "np2_40", "kw": {"np": 2, "max_levels": 40}},
    {"name": "nc2", "kw": {"nc": 2}},
    {"name": "variant2", "kw": {"variant": 2}},
    {"name": "variant5", "kw": {"variant": 5}},
    {"name": "ns0", "kw": {"ns": 0}},
    # each process's seen-set under a 3 MiB HBM budget (shard.hip spill_*)
    {"name": "seen_spill", "kw": {"seen_hbm_bytes": 3 << 20}},
    {"name": "np2_40_seen_spill", "kw": {"np": 2, "max_levels": 40, "seen_hbm_bytes": 16 << 20}},
    {"name": "lost_update", "kw": {"variant": 1, "invariants": 7}},
    {"name": "fault_pack", "kw": {}, "env": {"KC_FAULT": "1:7:1"}, "all_ranks": True},
    {"name": "fault_expand_hostrows", "kw": {}, "env": {"KC_FAULT": "0:9:0", "KC_DEVROW": "0"}, "all_ranks": True},
    # a failure after the all-gather, as if the exchange buffers could not be
    # grown: the rank still takes part in the exchange through its sink
    {"name": "fault_grow", "kw": {}, "env": {"KC_FAULT": "1:7:3"}, "all_ranks": True},
    # a failure found at the end of a narrow batch (sn_end) on one rank: the
    # failed process follows its peers into the next batch, whose first level
    # stops every rank (it used to leave for the gather alone)
    {"name": "fault_narrow_end", "kw": {}, "env": {"KC_FAULT": "1:12:4"}, "all_ranks": True},
    # round 5: every level on the counted path, so every level after the
    # first is a deferred frontier and its records go through the staging
    # segments across processes
    {"name": "model1_counted", "kw": {}, "env": {"KC_SNARROW": "0"}},
    {"name": "lost_update_counted", "kw": {"variant": 1, "invariants": 7}, "env": {"KC_SNARROW": "0"}},
    {"name": "np2_lost_update", "kw": {"np": 2, "variant": 1, "invariants": 7}},
    # round 5: TLC-ordered claims (ModelConfig.tlc_order): traces equal the oracle's
    {"name": "model1_tlc", "kw": {"tlc_order": True}},
    {"name": "nc2_tlc", "kw": {"nc": 2, "tlc_order": True}},
    {"name": "variant2_tlc", "kw": {"variant": 2, "tlc_order": True}},
    {"name": "variant3_tlc", "kw": {"variant": 3, "tlc_order": True}},
    {"name": "ns0_tlc", "kw": {"ns": 0, "tlc_order": True}},
    {"name": "lost_update_tlc", "kw": {"variant": 1, "invariants": 7, "tlc_order": True}},
    # round 6: first-claim claims (ModelConfig.first_claim) across processes
    {"name": "model1_first", "kw": {"first_claim": True}},
    {"name": "model1_first_counted", "kw": {"first_claim": True}, "env": {"KC_SNARROW": "0"}},
    {"name": "np2_40_first", "kw": {"np": 2, "max_levels": 40, "first_claim": True}},
    {"name": "nc2_first", "kw": {"nc": 2, "first_claim": True}, "env": {"KC_SNARROW": "0"}},
    {"name": "variant2_first", "kw": {"variant": 2, "first_claim": True}, "env": {"KC_SNARROW": "0"}},
    {"name": "ns0_first", "kw": {"ns": 0, "first_claim": True}},
    {"name": "lost_update_first", "kw": {"variant": 1, "invariants": 7, "first_claim": True},
     "env": {"KC_SNARROW": "0"}},
    {"name": "fault_first", "kw": {"first_claim": True}, "env": {"KC_FAULT": "1:7:2", "KC_SNARROW": "0"},
     "all_ranks": True},
]


def run_ranks(world, tmp_path):
    spec = tmp_path / "cases.json"
    spec.write_text(json.dumps(CASES))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.join(ROOT, "tests", "hostcomm_worker.py"), str(spec)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    out = {}
    dec = json.JSONDecoder()
    for line in p.stdout.splitlines():
        # (a line may hold more than one rank's record if their writes interleave)
        for chunk in line.split("RESULT ")[1:]:
            r, _ = dec.raw_decode(chunk)
            out.setdefault(r["case"], {})[r["rank"]] = r
    return out


@pytest.fixture(scope="module", params=[2, 3])
def results(request, tmp_path_factory):
    return request.param, run_ranks(request.param, tmp_path_factory.mktemp(f"hc{request.param}"))


def test_model1_exact(results, fixtures):
    world, res = results
    fx = fixtures["model1"]
    for name in ("model1", "model1_hostrows", "model1_pieces"):
        r = res[name][0]
        assert "exception" not in r, r.get("exception")
        assert r["complete"] and r["error"] is None and r["world"] == world
        assert r["level_width"] == fx["level_width"], name
        assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
        assert r["act_gen"] == fx["act_gen"]
        assert r["records_sent"] > 0          # records really crossed processes


def test_seen_spill_exact(results, fixtures):
    world, res = results
    fx = fixtures["model1"]
    r = res["seen_spill"][0]
    assert "exception" not in r, r.get("exception")
    assert r["complete"] and r["level_width"] == fx["level_width"]
    assert (r["distinct"], r["generated"]) == (fx["distinct"], fx["generated"])
    assert r["seen_flushes"] >= world and r["seen_cold_hits"] > 0


def test_np2_prefix_exact(results, fixtures):
    _, res = results
    fx = fixtures["np2_40levels"]
    for name in ("np2_40", "np2_40_seen_spill"):
        r = res[name][0]
        assert "exception" not in r, r.get("exception")
        assert r["level_width"] == fx["level_width"] and not r["complete"], name
        assert r["act_gen"] == fx["act_gen"], name
    assert res["np2_40_seen_spill"][0]["seen_flushes"] >= 2


@pytest.mark.parametrize("key,name,kind", [("nc2", "nc2", "assertion"), ("variant2", "variant2", "invariant"),
                                           ("variant5", "variant5", "invariant"), ("ns0", "ns0", "deadlock"),
                                           ("variant1_lost_update", "lost_update", "invariant")])
def test_errors_and_traces(results, fixtures, oracle, key, name, kind):
    _, res = results
    fx = fixtures[key]
    r = res[name][0]
    assert r["error"] == kind
    assert (r["error_level"], r["trace_len"]) == (fx["err_level"], fx["trace_len"])
    if kind == "assertion":
        assert r["error_action"] == fx["err_action"]
    if name == "lost_update":
        assert r["error_invariant"] == "NoLostUpdate"
    if name == "variant5":       # the first Init state in TLC's order, whichever rank owns it
        assert r["trace"] == fx["trace"]
    # the walk-back crossed ranks (broadcast); the trace is a real behaviour
    kw = {"nc2": dict(nc=2), "ns0": dict(ns=0)}.get(name, {})
    cfg = oracle.config(nc=kw.get("nc", 1), ns=kw.get("ns", 1),
                        variant={"variant2": 2, "variant5": 5, "lost_update": 1}.get(name, 0),
                        invariants=7 if name == "lost_update" else 3)
    for a, b in zip(r["trace"], r["trace"][1:]):
        succ, _ = oracle.successors(cfg, a)
        assert any(list(map(int, x)) == b for _, x in succ)


def test_tlc_order_traces(results, fixtures):
    _, res = results
    fx = fixtures["model1"]
    r = res["model1_tlc"][0]
    assert "exception" not in r, r.get("exception")
    assert r["complete"] and r["level_width"] == fx["level_width"]
    assert r["act_gen"] == fx["act_gen"] and r["act_dist"] == fx["act_dist"]
    for key, name, kind in (("nc2", "nc2_tlc", "assertion"), ("variant2", "variant2_tlc", "invariant"),
                            ("variant3", "variant3_tlc", "assertion"), ("ns0", "ns0_tlc", "deadlock"),
                            ("variant1_lost_update", "lost_update_tlc", "invariant")):
        r = res[name][0]
        assert "exception" not in r, (name, r.get("exception"))
        assert r["error"] == kind, name
        assert (r["error_level"], r["trace_len"]) == (fixtures[key]["err_level"], fixtures[key]["trace_len"]), name
        assert r["trace"] == fixtures[key]["trace"], name


def test_deferred_counted_levels(results, fixtures):
    _, res = results
    fx = fixtures["model1"]
    r = res["model1_counted"][0]
    assert "exception" not in r, r.get("exception")
    assert r["complete"] and r["level_width"] == fx["level_width"]
    assert (r["distinct"], r["generated"]) == (fx["distinct"], fx["generated"])
    assert r["act_gen"] == fx["act_gen"]
    assert sum(r["act_dist"].values()) + r["init"] == r["distinct"]
    for name, key in (("lost_update_counted", "variant1_lost_update"), ("np2_lost_update", "np2_variant1_lost_update")):
        r, fk = res[name][0], fixtures[key]
        assert "exception" not in r, r.get("exception")
        assert r["error"] == "invariant" and r["error_invariant"] == "NoLostUpdate", name
        assert (r["error_level"], r["trace_len"]) == (fk["err_level"], fk["trace_len"]), name


def test_first_claim(results, fixtures, oracle):
    # first-claim claims over gloo: counts exact, every error at the fixture's
    # level with a trace of the fixture's length that is a real behaviour
    world, res = results
    fx = fixtures["model1"]
    for name in ("model1_first", "model1_first_counted"):
        r = res[name][0]
        assert "exception" not in r, (name, r.get("exception"))
        assert r["claim_mode"] == "first" and r["complete"] and r["level_width"] == fx["level_width"], name
        assert (r["distinct"], r["generated"]) == (fx["distinct"], fx["generated"]) and r["act_gen"] == fx["act_gen"]
        assert sum(r["act_dist"].values()) + r["init"] == r["distinct"]
    r, fk = res["np2_40_first"][0], fixtures["np2_40levels"]
    assert "exception" not in r, r.get("exception")
    assert r["level_width"] == fk["level_width"] and r["act_gen"] == fk["act_gen"]
    for key, name, kind, kw in (("nc2", "nc2_first", "assertion", dict(nc=2)),
                                ("variant2", "variant2_first", "invariant", dict(variant=2)),
                                ("ns0", "ns0_first", "deadlock", dict(ns=0)),
                                ("variant1_lost_update", "lost_update_first", "invariant",
                                 dict(variant=1, invariants=7))):
        r, fk = res[name][0], fixtures[key]
        assert "exception" not in r, (name, r.get("exception"))
        assert r["error"] == kind, name
        assert (r["error_level"], r["trace_len"]) == (fk["err_level"], fk["trace_len"]), name
        cfg = oracle.config(nc=kw.get("nc", 1), ns=kw.get("ns", 1), variant=kw.get("variant", 0),
                            invariants=kw.get("invariants", 3))
        for a, b in zip(r["trace"], r["trace"][1:]):
            succ, _ = oracle.successors(cfg, a)
            assert any(list(map(int, x)) == b for _, x in succ), name
    got = res["fault_first"]
    assert sorted(got) == list(range(world))
    for rk, r in got.items():
        assert "exception" in r and ("injected fault" in r["exception"] or "failed" in r["exception"])


def test_fault_stops_every_rank(results):
    world, res = results
    for name in ("fault_pack", "fault_expand_hostrows", "fault_grow", "fault_narrow_end"):
        got = res[name]
        assert sorted(got) == list(range(world)), name
        for rk, r in got.items():
            assert "exception" in r, (name, rk)
            assert "injected fault" in r["exception"] or "failed" in r["exception"], r["exception"]
