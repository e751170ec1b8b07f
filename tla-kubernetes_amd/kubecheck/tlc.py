"""TLC-style command line for the KubeAPI model checker.

    python -m kubecheck.tlc [-config MC.cfg] [-deadlock] [-tool] [-nc N -np N -ns N]
                            [-variant V] [-workers N] [-fp K] [MC]

Reads the same inputs as the reference's toolbox run: a TLC model config
(KubeAPI.toolbox/Model_1/MC.cfg:1-16 — CONSTANT assignments, either direct
`X = TRUE` or TLC's `X <- def` indirection resolved through MC.tla:5-12;
SPECIFICATION; INVARIANT) and prints TLC's `-tool` message stream
(@!@!@STARTMSG code:class ... @!@!@ENDMSG code) for the messages the
reference run shows (MC.out: 2262, 2187, 2185, 2189/2190, 2193 with both
collision estimates, 2201/2773/2772/2202 coverage with TLC's source spans,
2200 progress, 2199, 2194, 2268 outdegree, 2186) plus violation reports.
SANY's messages (2220/2219) and expression-level coverage (2221) are not
produced (no TLA+ front end).  The model check itself
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
# build-defined (not in KubeAPI.tla): no Update overwrites a version its
# writer has not read (the optimistic concurrency HasRead gives Update,
# :733), with its lostUpdate history variable; run with -variant 1 it fails
BUILD_INVARIANTS = ("NoLostUpdate",)
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
    bad = [x for x in cfg["invariants"] if x not in KNOWN_INVARIANTS + BUILD_INVARIANTS]
    if bad:
        raise CfgError(f"unknown invariant(s) {bad}; KubeAPI.tla defines {KNOWN_INVARIANTS}"
                       f" (and the build {BUILD_INVARIANTS})")
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
    # the INVARIANT list selects the checks (an empty list checks none, as in TLC)
    kw["invariants"] = (1 if "TypeOK" in cfg["invariants"] else 0) | \
        (2 if "OnlyOneVersion" in cfg["invariants"] else 0) | \
        (4 if "NoLostUpdate" in cfg["invariants"] else 0)
    return kw


def msg(code: int, text: str, cls: int = 0, tool: bool = True) -> str:
    if not tool:
        return text
    return f"@!@!@STARTMSG {code}:{cls} @!@!@\n{text}\n@!@!@ENDMSG {code} @!@!@"


# Source locations TLC's coverage messages print for each action (msg 2772)
# and for Init (msg 2773): the definition heads in KubeAPI.tla, e.g.
# "DoRequest(self) ==" at KubeAPI.tla:471, columns 1-15 (MC.out:78-621, :48).
INIT_SPAN = (455, 1, 455, 4)
ACTION_SPANS = {
    "DoRequest": (471, 1, 471, 15), "DoReply": (485, 1, 485, 13),
    "DoListRequest": (499, 1, 499, 19), "DoListReply": (513, 1, 513, 17),
    "CStart": (528, 1, 528, 12), "C1": (551, 1, 551, 8), "C10": (558, 1, 558, 9),
    "C11": (570, 1, 570, 9), "c12": (577, 1, 577, 9), "C13": (589, 1, 589, 9),
    "C2": (596, 1, 596, 8), "C3": (604, 1, 604, 8), "C8": (611, 1, 611, 8),
    "C6": (618, 1, 618, 8), "C7": (631, 1, 631, 8), "C4": (638, 1, 638, 8),
    "C5": (645, 1, 645, 8), "PVCStart": (655, 1, 655, 14), "PVCListedPVCs": (665, 1, 665, 19),
    "PVCHavePVCs": (673, 1, 673, 17), "PVCDone": (690, 1, 690, 13), "APIStart": (698, 1, 698, 14),
}


def span_text(name: str, span) -> str:
    l1, c1, l2, c2 = span
    return f"<{name} line {l1}, col {c1} to line {l2}, col {c2} of module KubeAPI>"


def outdegree_stats(hist) -> Optional[tuple]:
    """(average, minimum, maximum, 95th percentile) of TLC's outdegree (new
    states first reached from an expanded state) from a 16-bin histogram
    (the last bin holds 15 or more)."""
    total = sum(hist)
    if not total:
        return None
    avg = sum(k * v for k, v in enumerate(hist)) / total
    lo = min(k for k, v in enumerate(hist) if v)
    hi = max(k for k, v in enumerate(hist) if v)
    acc, p95 = 0, hi
    for k, v in enumerate(hist):
        acc += v
        if acc >= 0.95 * total:
            p95 = k
            break
    return round(avg), lo, hi, p95


def java_e(x: float) -> str:
    """TLC's rendering of a probability: one decimal, exponent without
    padding (MC.out:41-42 "3.7E-9", "9.9E-10")."""
    m, e = f"{x:.1E}".split("E")
    return f"{m}E{int(e)}"


def tstamp(t: float) -> str:
    return time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(t))


def messages(r, t_start: float, t_end: float, actual_fp_prob: Optional[float] = None,
             engine: str = "", ngpus: int = 1) -> List[tuple]:
    """TLC -tool messages (code, class, body) for one check's result, in the
    order of the reference run (MC.out:1-1108).  SANY's (2220/2219) and the
    expression-level coverage (2221) are not produced: there is no TLA+ front
    end here."""
    out = []
    add = lambda code, text, cls=0: out.append((code, cls, text))  # noqa: E731
    add(2262, f"kubecheck (TLC-compatible counts) {engine}".rstrip())
    add(2187, f"Running breadth-first search Model-Checking with {ngpus} MI355X GPU(s) "
              f"(kubecheck ClaimSet FPSet, HBM StateQueue).")
    add(2185, f"Starting... ({tstamp(t_start)})")
    add(2189, "Computing initial states...")
    add(2190, f"Finished computing initial states: {r.init} distinct states generated at {tstamp(t_start)}.")
    d, g = r.distinct, r.generated
    minutes = max(t_end - t_start, 1e-9) / 60.0
    if r.error is None:
        body = ("Model checking completed. No error has been found.\n"
                "  Estimates of the probability that TLC did not check all reachable states\n"
                "  because two distinct states had the same fingerprint:\n"
                f"  calculated (optimistic):  val = {java_e(d * (g - d) / 2**64)}")
        if actual_fp_prob is not None:
            body += f"\n  based on the actual fingerprints:  val = {java_e(actual_fp_prob)}"
        add(2193, body)
    else:
        if r.error == "invariant":
            add(2110, f"Invariant {r.error_invariant} is violated.", 1)
        elif r.error == "assertion":
            add(2132, f"The first argument of Assert evaluated to FALSE (action {r.error_action}).", 1)
        else:
            add(2114, "Deadlock reached.", 1)
        add(2121, "The behavior up to this point is:", 1)
        blocks = re.split(r"^State (\d+):$", r.trace_text, flags=re.M)[1:]
        for num, body in zip(blocks[0::2], blocks[1::2]):
            add(2217, f"{num}: {body.strip()}", 4)
    add(2201, f"The coverage statistics at {tstamp(t_end)}")
    add(2773, f"{span_text('Init', INIT_SPAN)}: {r.init}:{r.init}")
    for name, span in ACTION_SPANS.items():
        add(2772, f"{span_text(name, span)}: {r.act_dist[name]}:{r.act_gen[name]}")
    add(2202, "End of statistics.")
    add(2200, f"Progress({r.depth}) at {tstamp(t_end)}: {g:,} states generated ({int(g / minutes):,} s/min), "
              f"{d:,} distinct states found ({int(d / minutes):,} ds/min), {r.queue_left:,} states left on queue.")
    add(2199, f"{g} states generated, {d} distinct states found, {r.queue_left} states left on queue.")
    add(2194, f"The depth of the complete state graph search is {r.depth}.")
    st = outdegree_stats(getattr(r, "outdeg_hist", []) or [])
    if st:
        add(2268, f"The average outdegree of the complete state graph is {st[0]} (minimum is {st[1]}, "
                  f"the maximum {st[2]} and the 95th percentile is {st[3]}).")
    add(2186, f"Finished in {int(round((t_end - t_start) * 1000))}ms at ({tstamp(t_end)})")
    return out


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
    ap.add_argument("-nocheckfps", action="store_true",
                    help="skip the 'based on the actual fingerprints' estimate (a sort of the seen-set)")
    a = ap.parse_args(argv)

    cfg_path = a.config or f"{a.spec}.cfg"
    if not os.path.exists(cfg_path):
        print(f"Error: cannot read model config {cfg_path}", file=sys.stderr)
        return 1
    tla_path = os.path.join(os.path.dirname(os.path.abspath(cfg_path)), f"{a.spec}.tla")
    defs = parse_defs(open(tla_path).read()) if os.path.exists(tla_path) else {}
    kw = model_from_cfg(parse_cfg(open(cfg_path).read(), defs))

    import kubecheck

    mc_cfg = kubecheck.ModelConfig(nc=a.nc, np=a.np, ns=a.ns, variant=a.variant, device=a.device,
                                   check_deadlock=not a.deadlock, **kw)
    t0 = time.time()
    with kubecheck.ModelChecker(mc_cfg) as mc:
        r = mc.run()
        prob = None if (a.nocheckfps or r.error is not None) else mc.check_fps()[1]
    t1 = t0 + r.seconds
    for code, cls, body in messages(r, t0, t1, prob, kubecheck.load().kc_build_info().decode(),
                                    kubecheck.device_count()):
        print(msg(code, body, cls, a.tool), flush=True)
    return 0 if r.error is None else 12


if __name__ == "__main__":
    sys.exit(main())
