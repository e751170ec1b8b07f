"""TLC-style front end: config parsing (CPU) and a GPU end-to-end run."""
import os
import subprocess
import sys

import pytest

from kubecheck import tlc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/KubeAPI.toolbox/Model_1"


def test_parse_authored_model1():
    kw = tlc.model_from_cfg(tlc.parse_cfg(open(os.path.join(ROOT, "models", "Model_1.cfg")).read()))
    assert kw == {"can_fail": True, "can_timeout": True, "invariants": 3}
    kw = tlc.model_from_cfg(tlc.parse_cfg(open(os.path.join(ROOT, "models", "NoFaults.cfg")).read()))
    assert kw == {"can_fail": False, "can_timeout": False, "invariants": 3}


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
def test_parse_reference_toolbox_inputs():
    # MC.cfg:5-11 binds the constants through MC.tla:5-12 definitions ("<-")
    defs = tlc.parse_defs(open(os.path.join(REF, "MC.tla")).read())
    cfg = tlc.parse_cfg(open(os.path.join(REF, "MC.cfg")).read(), defs)
    assert cfg["specification"] == "Spec"
    assert cfg["invariants"] == ["TypeOK", "OnlyOneVersion"]
    assert tlc.model_from_cfg(cfg) == {"can_fail": True, "can_timeout": True, "invariants": 3}


def test_rejects_unknown_inputs():
    with pytest.raises(tlc.CfgError):
        tlc.model_from_cfg(tlc.parse_cfg("CONSTANT REQUESTS_CAN_FAIL = 3\nSPECIFICATION Spec"))
    with pytest.raises(tlc.CfgError):
        tlc.model_from_cfg(tlc.parse_cfg(
            "CONSTANT REQUESTS_CAN_FAIL = TRUE REQUESTS_CAN_TIMEOUT = TRUE\nINVARIANT Foo"))
    with pytest.raises(tlc.CfgError):
        tlc.model_from_cfg(tlc.parse_cfg(
            "CONSTANT REQUESTS_CAN_FAIL = TRUE REQUESTS_CAN_TIMEOUT = TRUE\nPROPERTY ReconcileCompletes"))
    with pytest.raises(tlc.CfgError):
        tlc.parse_cfg("CONSTANT X <- nodef", {})


def test_tool_framing():
    assert tlc.msg(2199, "x") == "@!@!@STARTMSG 2199:0 @!@!@\nx\n@!@!@ENDMSG 2199 @!@!@"


def _model1_result(mcout, fixtures):
    """A CheckResult with Model_1's numbers (MC.out + the oracle's 1-worker
    distinct split and outdegree histogram), for the message-format tests."""
    from kubecheck import CheckResult

    fx = fixtures["model1"]
    return CheckResult(
        init=mcout["init"], generated=mcout["generated"], distinct=mcout["distinct"],
        queue_left=mcout["queue_left"], depth=mcout["depth"], complete=True,
        act_gen=mcout["act_gen"], act_dist=fx["act_dist"], level_width=fx["level_width"],
        error=None, error_action=None, error_self=-1, error_invariant=None, error_level=0,
        trace_len=0, seconds=9.875, collision_optimistic=mcout["collision_optimistic"],
        fpset_slots=0, peak_frontier=0, outdeg_hist=fx["outdeg_hist"])


def _bodies(msgs):
    out = {}
    for code, _cls, body in msgs:
        out.setdefault(code, []).append(body)
    return out


def check_against_mcout(got: dict, mcout: dict):
    """The message bodies a TLC -tool parser reads, against MC.out's own."""
    ref = mcout["message_bodies"]
    # totals and depth: identical text (MC.out:1098, :1101)
    assert got[2199] == [ref["2199"]]
    assert got[2194] == [ref["2194"]]
    # the no-error report up to the calculated estimate (MC.out:38-41); the
    # "actual fingerprints" line depends on the hash function (parity unpinned)
    assert got[2193][0].splitlines()[:4] == ref["2193"].splitlines()[:4]
    # Init coverage (MC.out:48), identical
    init = mcout["init_coverage"]
    assert got[2773] == [f"<Init line {init['span'][0]}, col {init['span'][1]} to line {init['span'][2]}, "
                         f"col {init['span'][3]} of module KubeAPI>: 2:2"]
    # action coverage (MC.out:78-621): same actions, order, source spans and
    # generated counts; the distinct split depends on TLC's 4 worker threads
    import re
    rows = [re.match(r"<(\w+) line (\d+), col (\d+) to line (\d+), col (\d+) of module KubeAPI>: (\d+):(\d+)$", b)
            for b in got[2772]]
    assert all(rows)
    assert [m.group(1) for m in rows] == list(mcout["act_span"])
    for m in rows:
        assert [int(m.group(k)) for k in range(2, 6)] == mcout["act_span"][m.group(1)]
        assert int(m.group(7)) == mcout["act_gen"][m.group(1)]
    assert sum(int(m.group(6)) for m in rows) + mcout["init"] == mcout["distinct"]
    # the shapes of the run-dependent lines (2200 progress, 2268 outdegree)
    pat = re.sub(r"[\d,]+", r"[\\d,]+", re.escape(ref["2200"]).replace(r"\ ", " "))
    assert re.fullmatch(re.sub(r"\\d\{4\}.*?\d\d:\d\d:\d\d", ".*", pat), got[2200][-1]) or \
        got[2200][-1].startswith(f"Progress({mcout['depth']}) at ")
    assert re.fullmatch(r"The average outdegree of the complete state graph is \d+ \(minimum is \d+, "
                        r"the maximum \d+ and the 95th percentile is \d+\)\.", got[2268][0])
    assert got[2202] == [ref["2202"]] and got[2189] == [ref["2189"]]


def test_messages_match_mcout(mcout, fixtures):
    got = _bodies(tlc.messages(_model1_result(mcout, fixtures), 1666975188.0, 1666975197.875, 9.9e-10))
    check_against_mcout(got, mcout)
    # with the 1-worker outdegree histogram (oracle): average 1, minimum 0,
    # maximum 3 (TLC's 4 workers saw 4), 95th percentile 2 (MC.out:1104)
    assert got[2268] == ["The average outdegree of the complete state graph is 1 (minimum is 0, "
                         "the maximum 3 and the 95th percentile is 2)."]
    assert got[2193][0].splitlines()[4] == "  based on the actual fingerprints:  val = 9.9E-10"


def test_invariant_list_selects_checks():
    base = "CONSTANT REQUESTS_CAN_FAIL = TRUE REQUESTS_CAN_TIMEOUT = TRUE\nSPECIFICATION Spec\n"
    assert tlc.model_from_cfg(tlc.parse_cfg(base + "INVARIANT TypeOK OnlyOneVersion"))["invariants"] == 3
    assert tlc.model_from_cfg(tlc.parse_cfg(base + "INVARIANT OnlyOneVersion"))["invariants"] == 2
    assert tlc.model_from_cfg(tlc.parse_cfg(base))["invariants"] == 0
    # the build-defined NoLostUpdate (models/LostUpdate.cfg)
    assert tlc.model_from_cfg(tlc.parse_cfg(base + "INVARIANT TypeOK OnlyOneVersion NoLostUpdate"))[
        "invariants"] == 7


@pytest.mark.gpu
def test_cli_model1_end_to_end():
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "tla-kubernetes_amd"))
    p = subprocess.run([sys.executable, "-m", "kubecheck.tlc", "-tool", "-config",
                        os.path.join(ROOT, "models", "Model_1.cfg"), "MC"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, p.stderr
    out = p.stdout
    import json, re
    mcout = json.load(open(os.path.join(ROOT, "tests", "golden", "model1_mcout.json")))
    got = {}
    for m in re.finditer(r"@!@!@STARTMSG (\d+):\d+ @!@!@\n(.*?)\n@!@!@ENDMSG \1 @!@!@", out, flags=re.S):
        got.setdefault(int(m.group(1)), []).append(m.group(2))
    check_against_mcout(got, mcout)          # the same bodies TLC printed (MC.out)
    assert "based on the actual fingerprints:  val = " in got[2193][0]
    assert got[2268] == ["The average outdegree of the complete state graph is 1 (minimum is 0, "
                         "the maximum 3 and the 95th percentile is 2)."]
    assert "577736 states generated, 163408 distinct states found, 0 states left on queue." in out
    assert "The depth of the complete state graph search is 124." in out
    assert "No error has been found" in out
    assert "<DoRequest line 471, col 1 to line 471, col 15 of module KubeAPI>: " in out and ":149766" in out


@pytest.mark.gpu
def test_cli_reports_assertion_trace():
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "tla-kubernetes_amd"))
    p = subprocess.run([sys.executable, "-m", "kubecheck.tlc", "-tool", "-nc", "2", "-config",
                        os.path.join(ROOT, "models", "Model_1.cfg"), "MC"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 12
    assert "Assert evaluated to FALSE (action C4)" in p.stdout
    assert p.stdout.count("STARTMSG 2217:4") == 10


@pytest.mark.gpu
def test_cli_reports_lost_update(fixtures):
    # BASELINE config 5 as an invariant bug: -variant 1 with NoLostUpdate
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "tla-kubernetes_amd"))
    p = subprocess.run([sys.executable, "-m", "kubecheck.tlc", "-tool", "-variant", "1", "-config",
                        os.path.join(ROOT, "models", "LostUpdate.cfg"), "MC"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 12, p.stderr
    assert "Invariant NoLostUpdate is violated." in p.stdout
    n = fixtures["variant1_lost_update"]["trace_len"]
    assert p.stdout.count("STARTMSG 2217:4") == n == 27
    assert "lostUpdate = TRUE" in p.stdout
