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
    assert kw == {"can_fail": True, "can_timeout": True}
    kw = tlc.model_from_cfg(tlc.parse_cfg(open(os.path.join(ROOT, "models", "NoFaults.cfg")).read()))
    assert kw == {"can_fail": False, "can_timeout": False}


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
def test_parse_reference_toolbox_inputs():
    # MC.cfg:5-11 binds the constants through MC.tla:5-12 definitions ("<-")
    defs = tlc.parse_defs(open(os.path.join(REF, "MC.tla")).read())
    cfg = tlc.parse_cfg(open(os.path.join(REF, "MC.cfg")).read(), defs)
    assert cfg["specification"] == "Spec"
    assert cfg["invariants"] == ["TypeOK", "OnlyOneVersion"]
    assert tlc.model_from_cfg(cfg) == {"can_fail": True, "can_timeout": True}


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


@pytest.mark.gpu
def test_cli_model1_end_to_end():
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "tla-kubernetes_amd"))
    p = subprocess.run([sys.executable, "-m", "kubecheck.tlc", "-tool", "-config",
                        os.path.join(ROOT, "models", "Model_1.cfg"), "MC"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, p.stderr
    out = p.stdout
    assert "577736 states generated, 163408 distinct states found, 0 states left on queue." in out
    assert "The depth of the complete state graph search is 124." in out
    assert "No error has been found" in out
    assert "<DoRequest>: " in out and ":149766" in out


@pytest.mark.gpu
def test_cli_reports_assertion_trace():
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "tla-kubernetes_amd"))
    p = subprocess.run([sys.executable, "-m", "kubecheck.tlc", "-tool", "-nc", "2", "-config",
                        os.path.join(ROOT, "models", "Model_1.cfg"), "MC"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 12
    assert "Assert evaluated to FALSE (action C4)" in p.stdout
    assert p.stdout.count("STARTMSG 2217:4") == 10
