"""The product's lowered spec (packed GPU layout, host-compiled from the same
kubeapi_spec.h the kernels use) against the CPU oracle, state by state.

Runs on CPU through kc_spec_* (no GPU, no BFS engine): every state of the
explored prefix must have the same successor list — same order, same action,
same canonical value — and the same invariant verdicts in both."""
import numpy as np
import pytest

from kubecheck import ModelConfig, Spec


def _bfs_compare(oracle, nc, np_, ns, max_levels=0, **flags):
    ocfg = oracle.config(nc, np_, ns, **flags)
    sp = Spec(ModelConfig(nc=nc, np=np_, ns=ns, **flags))
    init = sp.init()
    assert (init == oracle.level_tuples(ocfg, 1)).all()
    seen = {tuple(x) for x in init}
    frontier, level, checked, widths = list(init), 1, 0, []
    failure = None
    while frontier and (not max_levels or level <= max_levels):
        widths.append(len(frontier))
        nxt = []
        for s in frontier:
            ps, pf = sp.successors(s)
            os_, of = oracle.successors(ocfg, s)
            assert sp.fp_selfcheck(s) == 0      # kernels' incremental fingerprint
            assert pf == of
            checked += 1
            if ps is None:
                failure = failure or (level, pf)
                continue
            assert len(ps) == len(os_)
            for (a, x), (b, y) in zip(ps, os_):
                assert a == b and np.array_equal(x, y)
                k = tuple(x)
                if k not in seen:
                    seen.add(k)
                    assert sp.check_invariants(x) is None
                    nxt.append(x)
        frontier, level = nxt, level + 1
    return checked, widths, failure


def test_model1_full_state_space(oracle, fixtures):
    checked, widths, failure = _bfs_compare(oracle, 1, 1, 1)
    assert checked == 163408 and failure is None
    assert widths == fixtures["model1"]["level_width"]


@pytest.mark.parametrize("flags", [dict(can_fail=False, can_timeout=False),
                                   dict(can_fail=True, can_timeout=False)])
def test_model1_constant_variants(oracle, fixtures, flags):
    key = f"model1_fail{int(flags['can_fail'])}_timeout{int(flags['can_timeout'])}"
    checked, widths, _ = _bfs_compare(oracle, 1, 1, 1, **flags)
    assert widths == fixtures[key]["level_width"]


def test_two_clients_seeded_bug(oracle, fixtures):
    _, widths, failure = _bfs_compare(oracle, 2, 1, 1, max_levels=10)
    assert widths == fixtures["nc2"]["level_width"]
    assert failure == (10, "C4")


def test_two_servers_and_two_controllers(oracle, fixtures):
    _, widths, _ = _bfs_compare(oracle, 1, 1, 2, max_levels=30)
    assert widths == fixtures["ns2"]["level_width"][:30]
    _, widths, _ = _bfs_compare(oracle, 1, 2, 1, max_levels=9)
    assert widths == fixtures["np2_40levels"]["level_width"][:9]


def test_pack_roundtrip_and_fingerprint_canonical(oracle):
    sp = Spec(ModelConfig())
    cfg = oracle.config()
    fps = {}
    for level in (5, 40, 90):
        for t in oracle.level_tuples(cfg, level)[:500]:
            p = sp.pack(t)
            assert np.array_equal(sp.unpack(p), t)
            fp = sp.fingerprint(t)
            assert 0 < fp < 2**63
            assert fps.setdefault(fp, tuple(t)) == tuple(t)   # no collisions in the sample


def test_tuple_outside_domain_rejected():
    sp = Spec(ModelConfig())
    bad = sp.init()[0].copy()
    bad[0] = 1 << 40                                          # apiState bit beyond |U|
    with pytest.raises(Exception):
        sp.successors(bad)


def test_lost_update_ghost_matches_oracle(oracle, fixtures):
    # variant 1 (Update without HasRead, KubeAPI.tla:733) with the
    # build-defined NoLostUpdate: the lostUpdate history variable and its
    # successors agree with the oracle state by state up to the level before
    # the violation, and the oracle's counterexample replays through the
    # product's spec, ending in the state that breaks NoLostUpdate
    _, widths, failure = _bfs_compare(oracle, 1, 1, 1, max_levels=25, variant=1, invariants=7)
    fx = fixtures["variant1_lost_update"]
    assert widths == fx["level_width"][:25] and failure is None
    sp = Spec(ModelConfig(variant=1, invariants=7))
    tr = [np.array(t, dtype=np.uint64) for t in fx["trace"]]
    for a, b in zip(tr, tr[1:]):
        succ, _ = sp.successors(a)
        assert any(np.array_equal(x, b) for _, x in succ)
        assert sp.check_invariants(a) is None
    assert sp.check_invariants(tr[-1]) == "NoLostUpdate"
    assert int(tr[-1][0]) >> 63 == 1                          # lostUpdate: bit 63 of the apiState word
    # without the check the ghost does not exist: the same Update leaves no trace
    plain = Spec(ModelConfig(variant=1))
    succ, _ = plain.successors(tr[-2])
    assert all(int(x[0]) >> 63 == 0 for _, x in succ)
