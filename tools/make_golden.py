#!/usr/bin/env python3
"""Generate tests/golden fixtures.

1. tests/golden/model1_mcout.json — numbers extracted from the reference's
   recorded TLC run, /root/reference/KubeAPI.toolbox/Model_1/MC.out (data
   only: counts and the MC.out line each came from).  Needs /root/reference.
2. tests/golden/oracle_fixtures.json — results of the CPU oracle (itself
   pinned by (1)) for the parameterised variants: level widths, per-action
   distinct counts under sequential BFS order, the NC=2 seeded-bug trace.

Usage: python tools/make_golden.py [--mcout] [--oracle] [--np2]
"""
from __future__ import annotations

import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
MCOUT = "/root/reference/KubeAPI.toolbox/Model_1/MC.out"

# MC.out coverage lines -> oracle branch / coverage counter names.  Each key
# is the "line L, col C to line L2, col C2" span TLC prints (msg 2221).
SPANS = {
    "cov.api": (778, 27, 778, 45),            # \A o \in apiState body: sum |apiState|
    "cov.req": (780, 34, 780, 60),            # sum |DOMAIN requests|
    "cov.lreq": (781, 38, 781, 72),           # sum |DOMAIN listRequests|
    "cov.objs": (434, 25, 435, 39),           # sum |objs|
    "cov.api2": (788, 29, 789, 51),           # sum |apiState|^2
    "branch.CSTART_THEN": (533, 28, 541, 42),
    "branch.CSTART_ELSE": (542, 31, 546, 82),
    "branch.C1_START": (553, 24, 553, 62),
    "branch.C1_C10": (554, 24, 554, 59),
    "branch.C11_START": (572, 25, 572, 63),
    "branch.C11_c12": (573, 25, 573, 60),
    "branch.C13_START": (591, 25, 591, 63),
    "branch.C13_C2": (592, 25, 592, 59),
    "branch.C3_START": (606, 24, 606, 62),
    "branch.C3_C8": (607, 24, 607, 58),
    "branch.C8_C4": (613, 24, 613, 58),
    "branch.C8_C6": (614, 24, 614, 58),
    "branch.C7_START": (633, 24, 633, 62),
    "branch.C7_C4": (634, 24, 634, 58),
    "branch.PVCL_START": (668, 35, 668, 75),
    "branch.PVCL_HAVE": (669, 35, 669, 78),
    "branch.API_CREATE": (702, 52, 702, 102),   # Create-exists branch (0) + 704 (0)
    "branch.API_FORCE": (707, 55, 707, 104),
    "branch.API_FORCE_REPLACE": (708, 63, 713, 91),
    "branch.API_FORCE_CREATE": (714, 60, 714, 114),
    "branch.API_GET": (717, 66, 717, 115),
    "branch.API_GET_NOTFOUND": (727, 74, 727, 124),
    "branch.API_DELETE": (730, 74, 730, 135),
    "branch.API_UPDATE": (733, 88, 733, 156),
    "branch.API_UPDATE_OK": (734, 96, 736, 131),
    "branch.API_UPDATE_ERR": (738, 96, 738, 146),
    "branch.API_LIST": (746, 33, 747, 88),
    "branch.API_ASSERT": (742, 85, 743, 108),
}


def parse_mcout(path: str) -> dict:
    text = open(path).read()
    lines = text.splitlines()
    out: dict = {"source": "KubeAPI.toolbox/Model_1/MC.out (TLC2 2.16 rev cdddf55)"}

    def where(pattern):
        for i, l in enumerate(lines, 1):
            if re.search(pattern, l):
                return i, l
        raise KeyError(pattern)

    i, l = where(r"states generated, .* distinct states found")
    m = re.search(r"([\d,]+) states generated, ([\d,]+) distinct states found, ([\d,]+) states left", l)
    out["generated"], out["distinct"], out["queue_left"] = (int(x.replace(",", "")) for x in m.groups())
    out["line_totals"] = i
    i, l = where(r"The depth of the complete state graph search is")
    out["depth"] = int(re.search(r"is (\d+)", l).group(1))
    out["line_depth"] = i
    i, l = where(r"Finished computing initial states")
    out["init"] = int(re.search(r"(\d+) distinct states generated", l).group(1))
    out["line_init"] = i
    out["no_error"] = "No error has been found" in text
    act_gen, act_dist, act_line, act_span = {}, {}, {}, {}
    for i, l in enumerate(lines, 1):
        m = re.match(r"<(\w+) line (\d+), col (\d+) to line (\d+), col (\d+) of module KubeAPI>: (\d+):(\d+)", l)
        if not m:
            continue
        span = [int(m.group(k)) for k in range(2, 6)]
        if m.group(1) == "Init":                     # msg 2773, Init's own line
            out["init_coverage"] = {"distinct": int(m.group(6)), "generated": int(m.group(7)),
                                    "mcout_line": i, "span": span}
        else:
            act_dist[m.group(1)] = int(m.group(6))   # worker-order dependent
            act_gen[m.group(1)] = int(m.group(7))
            act_line[m.group(1)] = i
            act_span[m.group(1)] = span              # msg 2772's location of the action
    out["act_span"] = act_span
    out["act_gen"] = act_gen
    out["act_dist_tlc_4workers"] = act_dist
    out["act_line"] = act_line
    spans = {}
    for name, (l1, c1, l2, c2) in SPANS.items():
        pat = re.compile(rf"^\s*\|*line {l1}, col {c1} to line {l2}, col {c2} of module KubeAPI: (\d+)")
        for i, l in enumerate(lines, 1):
            m = pat.match(l)
            if m:
                spans[name] = {"value": int(m.group(1)), "mcout_line": i}
                break
        else:
            raise KeyError(name)
    out["spans"] = spans
    m = re.search(r"calculated \(optimistic\):\s+val = ([\dE.-]+)", text)
    out["collision_optimistic"] = float(m.group(1))
    # message bodies a TLC -tool parser reads (code -> body text), for the
    # CLI's message-format test; 2200/2268 values are run dependent
    bodies = {}
    for m in re.finditer(r"@!@!@STARTMSG (\d+):\d+ @!@!@\n(.*?)\n@!@!@ENDMSG \1 @!@!@", text, flags=re.S):
        code = int(m.group(1))
        if code in (2190, 2193, 2199, 2194, 2268, 2200, 2201, 2202, 2186, 2185, 2189):
            bodies.setdefault(str(code), m.group(2))
    out["message_bodies"] = bodies
    return out


def oracle_fixtures(with_np2: bool) -> dict:
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O

    O.build()
    fx: dict = {"generator": "tools/make_golden.py (oracle/kubeapi_oracle.c)"}

    def summary(r):
        out = {k: r[k] for k in ("init", "generated", "distinct", "depth", "complete", "act_gen",
                                 "act_dist", "level_width", "err_kind", "err_action", "err_self",
                                 "err_level", "trace_len")}
        # new states first reached per expanded state (TLC outdegree), 16 bins, last = 15+
        h = r["newdeg_hist"]
        out["outdeg_hist"] = h[:15] + [sum(h[15:])]
        return out

    fx["model1"] = summary(O.run(O.config()))
    for f, t in [(0, 0), (0, 1), (1, 0)]:
        fx[f"model1_fail{f}_timeout{t}"] = summary(O.run(O.config(can_fail=f, can_timeout=t)))
    r = O.run(O.config(nc=2))
    fx["nc2"] = summary(r)
    fx["nc2"]["trace"] = [[int(x) for x in t] for t in r["trace"]]
    fx["nc2_np0"] = summary(O.run(O.config(nc=2, np_=0)))
    r = O.run(O.config(variant=2))                       # Force without replace
    fx["variant2"] = summary(r)
    fx["variant2"]["err_invariant"] = r["err_invariant"]
    fx["variant2"]["trace"] = [[int(x) for x in t] for t in r["trace"]]
    fx["variant1"] = summary(O.run(O.config(variant=1)))  # Update without HasRead
    # the lost update as an invariant violation (SURVEY §8(d) config 5's
    # second variant): the build-defined NoLostUpdate (bit 2) with its
    # lostUpdate history variable; KubeAPI.tla as written keeps it (the
    # state space is Model_1's), variant 1 breaks it
    for key, cfg in (("variant1_lost_update", O.config(variant=1, invariants=7)),
                     ("np2_variant1_lost_update", O.config(np_=2, variant=1, invariants=7)),
                     ("nc2np0_variant1_lost_update", O.config(nc=2, np_=0, variant=1, invariants=7))):
        r = O.run(cfg)
        fx[key] = summary(r)
        fx[key]["err_invariant"] = r["err_invariant"]
        fx[key]["trace"] = [[int(x) for x in t] for t in r["trace"]]
    fx["model1_lost_update_checked"] = summary(O.run(O.config(invariants=7)))
    # seeded bugs that exercise the other error paths (kubeapi_spec.h Flags):
    # 3 = C2 Assert (KubeAPI.tla:598-599), 4 = TypeOK, 5 = Init violates
    # OnlyOneVersion; ns=0 (no API server) deadlocks (launch:16)
    for key, cfg in (("variant3", O.config(variant=3)), ("variant4", O.config(variant=4)),
                     ("variant5", O.config(variant=5)), ("ns0", O.config(ns=0))):
        r = O.run(cfg)
        fx[key] = summary(r)
        fx[key]["err_invariant"] = r["err_invariant"]
        fx[key]["trace"] = [[int(x) for x in t] for t in r["trace"]]
    fx["ns0_nodeadlock"] = summary(O.run(O.config(ns=0, check_deadlock=False)))
    # a .cfg INVARIANT list without one of the two: the seeded violation of
    # the unlisted invariant is not reported and the check runs to the end
    fx["variant4_oov_only"] = summary(O.run(O.config(variant=4, invariants=2)))
    fx["variant5_no_invariants"] = summary(O.run(O.config(variant=5, invariants=0)))
    fx["ns2"] = summary(O.run(O.config(ns=2)))
    fx["nc1_np0"] = summary(O.run(O.config(np_=0)))
    fx["np2_40levels"] = summary(O.run(O.config(np_=2, max_levels=40, keep_trace=False)))
    if with_np2:
        path = os.path.join(GOLDEN, "np2_full.json")
        if os.path.exists(path):
            fx["np2_full"] = json.load(open(path))
        # NP=3 (SURVEY §8(d) config 2 secondary): its first 40 levels, from
        # `kubeapi_oracle -np 3 -notracestore -maxlevels 40` (112 s)
        path = os.path.join(GOLDEN, "np3_40levels.json")
        if os.path.exists(path):
            fx["np3_40levels"] = json.load(open(path))
    return fx


def main() -> None:
    os.makedirs(GOLDEN, exist_ok=True)
    args = set(sys.argv[1:]) or {"--mcout", "--oracle"}
    if "--mcout" in args:
        g = parse_mcout(MCOUT)
        json.dump(g, open(os.path.join(GOLDEN, "model1_mcout.json"), "w"), indent=1)
        print("wrote model1_mcout.json")
    if "--oracle" in args:
        fx = oracle_fixtures("--np2" in args)
        json.dump(fx, open(os.path.join(GOLDEN, "oracle_fixtures.json"), "w"))
        print("wrote oracle_fixtures.json")


if __name__ == "__main__":
    main()
