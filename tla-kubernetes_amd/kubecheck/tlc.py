"""TLC-style command line for the KubeAPI model checker.

    python -m kubecheck.tlc [-config MC.cfg] [-deadlock] [-tool] [-nc N -np N -ns N]
                            [-variant V] [-workers N] [-fp K] [MC]

Reads the same inputs as the reference's toolbox run: a TLC model config
(KubeAPI.toolbox/Model_1/MC.cfg:1-16 — CONSTANT assignments, either direct
`X = TRUE` or TLC's `X <- def` indirection resolved through MC.tla:5-12;
SPECIFICATION; INVARIANT) and prints TLC's `-tool` message stream
(@!@!@STARTMSG code:class ... @!@!@ENDMSG code) for the messages the
reference run shows (MC.out: 2262, 2187, 2185, 2189/2190, 2193, 2201/2772/
2202, 2199, 2194, 2186) plus violation reports.  The model check itself
runs on the GPU (kubecheck.ModelChecker); -workers and -fp are accepted for
command-line compatibility (the GPU replaces the worker pool; fingerprints
are kubecheck's own 64-bit hash, not TLC's FP64 #K).
"""
from __future__ import annotations

import argparse
import os
import re
import sys
import time
from typing import Dict, List, Optional

KNOWN_INVARIANTS = ("TypeOK", "OnlyOneVersion")          # KubeAPI.tla:776,787
KNOWN_CONSTANTS = ("REQUESTS_CAN_FAIL", "REQUESTS_CAN_TIMEOUT", "defaultInitValue")  # :4-6,374


class CfgError(ValueError):
    pass


def _strip_comments(text: str) -> str:
    text = re.sub(r"\(\*.*?\*\)", " ", text, flags=re.S)
    return "\n".join(line.split("\\*", 1)[0] for line in text.splitlines())


def parse_defs(tla_text: str) -> Dict[str, str]:
    """`name == value` definitions of a TLC-generated MC.tla (MC.tla:5-12)."""
    out = {}
    for m in re.finditer(r"^(\w+)\s*==\s*\n?\s*(\S+)", _strip_comments(tla_text), flags=re.M):
        out[m.group(1)] = m.group(2)
    return out


def parse_cfg(cfg_text: str, defs: Optional[Dict[str, str]] = None) -> dict:
    """Parse a TLC .cfg (the subset MC.cfg uses)."""
    defs = defs or {}
    toks = _strip_comments(cfg_text).split()
    out: dict = {"constants": {}, "specification": None, "invariants": [], "properties": []}
    i, section = 0, None
    keywords = {"CONSTANT", "CONSTANTS", "SPECIFICATION", "INVARIANT", "INVARIANTS",
                "PROPERTY", "PROPERTIES", "INIT", "NEXT"}
    while i < len(toks):
        t = toks[i]
        if t in keywords:
            section = t
            i += 1
            continue
        if section in ("CONSTANT", "CONSTANTS"):
            if i + 2 < len(toks) + 1 and i + 1 < len(toks) and toks[i + 1] in ("=", "<-"):
                name, op, val = t, toks[i + 1], toks[i + 2]
                if op == "<-":
                    if val not in defs:
                        raise CfgError(f"{name} <- {val}: definition {val} not found in MC.tla")
                    val = defs[val]
                out["constants"][name] = val
                i += 3
                continue
            raise CfgError(f"bad CONSTANT entry near {t!r}")
        if section == "SPECIFICATION":
            out["specification"] = t
        elif section in ("INVARIANT", "INVARIANTS"):
            out["invariants"].append(t)
        elif section in ("PROPERTY", "PROPERTIES"):
            out["properties"].append(t)
        else:
            raise CfgError(f"unsupported cfg token {t!r}")
        i += 1
    return out


def model_from_cfg(cfg: dict) -> dict:
    """Validate a parsed cfg against KubeAPI.tla and map it to ModelConfig kwargs."""
    if cfg["specification"] not in (None, "Spec"):
        raise CfgError(f"SPECIFICATION {cfg['specification']}: only Spec (KubeAPI.tla:765)")
    bad = [x for x in cfg["invariants"] if x not in KNOWN_INVARIANTS]
    if bad:
        raise CfgError(f"unknown invariant(s) {bad}; KubeAPI.tla defines {KNOWN_INVARIANTS}")
    if cfg["properties"]:
        raise CfgError("temporal PROPERTY checking (liveness) is out of scope")
    kw = {}
    for name, key in (("REQUESTS_CAN_FAIL", "can_fail"), ("REQUESTS_CAN_TIMEOUT", "can_timeout")):
        v = cfg["constants"].get(name)
        if v not in ("TRUE", "FALSE"):
            raise CfgError(f"{name} must be TRUE or FALSE (ASSUME, KubeAPI.tla:8-9), got {v!r}")
        kw[key] = v == "TRUE"
    unknown = set(cfg["constants"]) - set(KNOWN_CONSTANTS)
    if unknown:
        raise CfgError(f"unknown CONSTANT(s) {sorted(unknown)}")
    if cfg["invariants"] and set(cfg["invariants"]) != set(KNOWN_INVARIANTS):
        raise CfgError("kubecheck always checks both TypeOK and OnlyOneVersion")
    return kw


def msg(code: int, text: str, cls: int = 0, tool: bool = True) -> str:
    if not tool:
        return text
    return f"@!@!@STARTMSG {code}:{cls} @!@!@\n{text}\n@!@!@ENDMSG {code} @!@!@"


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="kubecheck.tlc", description=__doc__.split("\n\n")[0])
    ap.add_argument("spec", nargs="?", default="MC")
    ap.add_argument("-config", default=None)
    ap.add_argument("-deadlock", action="store_true", help="do NOT check for deadlock (TLC flag)")
    ap.add_argument("-tool", action="store_true")
    ap.add_argument("-workers", default="1")
    ap.add_argument("-fp", type=int, default=None)
    ap.add_argument("-nc", type=int, default=1)
    ap.add_argument("-np", type=int, default=1)
    ap.add_argument("-ns", type=int, default=1)
    ap.add_argument("-variant", type=int, default=0)
    ap.add_argument("-device", type=int, default=0)
    a = ap.parse_args(argv)

    cfg_path = a.config or f"{a.spec}.cfg"
    if not os.path.exists(cfg_path):
        print(f"Error: cannot read model config {cfg_path}", file=sys.stderr)
        return 1
    tla_path = os.path.join(os.path.dirname(os.path.abspath(cfg_path)), f"{a.spec}.tla")
    defs = parse_defs(open(tla_path).read()) if os.path.exists(tla_path) else {}
    kw = model_from_cfg(parse_cfg(open(cfg_path).read(), defs))

    import kubecheck

    out = lambda code, text, cls=0: print(msg(code, text, cls, a.tool), flush=True)  # noqa: E731
    out(2262, f"kubecheck (TLC-compatible counts) {kubecheck.load().kc_build_info().decode()}")
    mc_cfg = kubecheck.ModelConfig(nc=a.nc, np=a.np, ns=a.ns, variant=a.variant, device=a.device,
                                   check_deadlock=not a.deadlock, **kw)
    out(2187, f"Running breadth-first search Model-Checking on {kubecheck.device_count()} "
              f"MI355X GPU(s) (HBM FPSet, HBM StateQueue) for {mc_cfg.name}.")
    out(2185, f"Starting... ({time.strftime('%Y-%m-%d %H:%M:%S')})")
    out(2189, "Computing initial states...")
    with kubecheck.ModelChecker(mc_cfg) as mc:
        r = mc.run()
    out(2190, f"Finished computing initial states: {r.init} distinct states generated.")
    rc = 0
    if r.error is None:
        d, g = r.distinct, r.generated
        out(2193, "Model checking completed. No error has been found.\n"
                  "  Estimates of the probability that TLC did not check all reachable states\n"
                  "  because two distinct states had the same fingerprint:\n"
                  f"  calculated (optimistic):  val = {d * (g - d) / 2**64:.1E}")
    else:
        rc = 12
        if r.error == "invariant":
            out(2110, f"Invariant {r.error_invariant} is violated.", 1)
        elif r.error == "assertion":
            out(2132, f"The first argument of Assert evaluated to FALSE (action {r.error_action}).", 1)
        else:
            out(2114, "Deadlock reached.", 1)
        out(2121, "The behavior up to this point is:", 1)
        blocks = re.split(r"^State (\d+):$", r.trace_text, flags=re.M)[1:]
        for num, body in zip(blocks[0::2], blocks[1::2]):
            out(2217, f"{num}: {body.strip()}", 4)
    out(2201, "The coverage statistics:")
    for name in kubecheck.ACTIONS:
        out(2772, f"<{name}>: {r.act_dist[name]}:{r.act_gen[name]}")
    out(2202, "End of statistics.")
    out(2199, f"{r.generated} states generated, {r.distinct} distinct states found, "
              f"{r.queue_left} states left on queue.")
    out(2194, f"The depth of the complete state graph search is {r.depth}.")
    out(2186, f"Finished in {int(r.seconds * 1000)}ms at ({time.strftime('%Y-%m-%d %H:%M:%S')})")
    return rc


if __name__ == "__main__":
    sys.exit(main())
