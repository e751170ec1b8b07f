"""Pin the CPU oracle against the reference's own recorded TLC run
(KubeAPI.toolbox/Model_1/MC.out) before trusting it for anything else."""
import pytest


@pytest.fixture(scope="module")
def model1(oracle):
    return oracle.run(oracle.config())


def test_totals(model1, mcout):
    # MC.out:32 (init), :1098 (generated/distinct/left), :1101 (depth), :38 (no error)
    assert model1["init"] == mcout["init"] == 2
    assert model1["generated"] == mcout["generated"] == 577736
    assert model1["distinct"] == mcout["distinct"] == 163408
    assert model1["queue_left"] == mcout["queue_left"] == 0
    assert model1["depth"] == mcout["depth"] == 124
    assert mcout["no_error"] and model1["err_kind"] == 0 and model1["complete"]


def test_per_action_generated(model1, mcout):
    # MC.out:78-621, msg 2772 "<Action ...>: distinct:generated"; generated is
    # deterministic, the distinct split depends on TLC's 4 worker threads.
    assert model1["act_gen"] == mcout["act_gen"]
    assert sum(model1["act_dist"].values()) + model1["init"] == model1["distinct"]


def test_coverage_sums(model1, mcout):
    # TypeOK / OnlyOneVersion sub-expression counts, MC.out:1029-1080
    for k in ("api", "req", "lreq", "objs", "api2"):
        assert model1["cov"][k] == mcout["spans"]["cov." + k]["value"], k


def test_branch_counts(model1, mcout):
    # every IF/CASE branch count TLC recorded for Next's actions
    for name, rec in mcout["spans"].items():
        if name.startswith("branch."):
            assert model1["branch"][name[7:]] == rec["value"], (name, rec)


def test_collision_estimate(model1, mcout):
    # TLC's optimistic estimate d*(g-d)/2^64 (MC.out:41)
    d, g = model1["distinct"], model1["generated"]
    assert f"{d * (g - d) / 2**64:.1E}" == f"{mcout['collision_optimistic']:.1E}"


def test_oracle_fixtures_reproduce(oracle, fixtures):
    # the committed oracle fixtures are what the oracle computes now
    r = oracle.run(oracle.config(nc=2))
    fx = fixtures["nc2"]
    for k in ("distinct", "generated", "level_width", "err_kind", "err_action", "err_level",
              "trace_len"):
        assert r[k] == fx[k], k
    assert [list(map(int, t)) for t in r["trace"]] == fx["trace"]
    assert fixtures["model1"]["level_width"][:12] == [2, 4, 10, 16, 25, 35, 43, 52, 57, 64, 68, 74]


def test_seeded_bug_is_c4_assert(fixtures):
    # two clients sharing Secret/foo -> C4
    # Assert(~ObjectExists(Secret)) (KubeAPI.tla:639-640) fails at depth 10
    fx = fixtures["nc2"]
    assert fx["err_kind"] == 1 and fx["err_action"] == "C4"
    assert fx["err_level"] == 10 and fx["trace_len"] == 10
    assert fx["level_width"] == [4, 12, 36, 76, 148, 256, 406, 611, 859, 1171]


def test_constants_false_variants(oracle, fixtures):
    for f, t in [(0, 0), (0, 1), (1, 0)]:
        r = oracle.run(oracle.config(can_fail=f, can_timeout=t))
        fx = fixtures[f"model1_fail{f}_timeout{t}"]
        assert (r["distinct"], r["generated"], r["depth"]) == (fx["distinct"], fx["generated"], fx["depth"])
    # REQUESTS_CAN_FAIL only adds duplicate Error branches when TIMEOUT is on
    assert fixtures["model1_fail0_timeout1"]["distinct"] == 163408


def test_successor_semantics_spot(oracle):
    # DoRequest yields 3 successors when both constants are TRUE (KubeAPI.tla:472-480):
    # Pending, then Error twice (the constant disjunction branches).
    cfg = oracle.config()
    init = oracle.level_tuples(cfg, 1)
    succ, fail = oracle.successors(cfg, init[1])        # shouldReconcile = TRUE
    assert fail is None and [a for a, _ in succ] == ["CStart", "CStart", "PVCStart"]
    s = succ[0][1]
    succ2, _ = oracle.successors(cfg, s)
    assert [a for a, _ in succ2] == ["DoRequest"] * 3 + ["PVCStart"]


def test_parallel_comparator_counts(mcout, oracle):
    # the multi-core CPU comparator (bench.py cpu_baseline) explores the same
    # state space: MC.out's totals (MC.out:1098) on 1 and 4 threads
    for threads in (1, 4):
        cfg = oracle.config(keep_trace=False)
        cfg.fpset_log2 = 22
        r = oracle.bench_parallel(cfg, threads, 60.0)
        assert r["complete"] and not r["set_full"]
        assert (r["distinct"], r["generated"], r["levels"]) == (
            mcout["distinct"], mcout["generated"], mcout["depth"])
