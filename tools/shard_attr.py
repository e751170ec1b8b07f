"""Per-rank, per-kernel attribution of an emulated sharded NP=2 check
(VERDICT r4 "next" item 1a).

  run:        python tools/shard_attr.py run R [--checks K] [--tlc | --first]
              K (default 2) sharded NP=2 checks with R ranks emulated on one
              GPU; with KC_SERIAL=1 in the environment every rank's stage is
              synchronised before the next rank's launches, so no two ranks'
              kernels overlap.  Prints one JSON line per check (wall ms,
              distinct).  Run it under rocprofv3 --kernel-trace.  --tlc:
              with ModelConfig.tlc_order (TLC-ordered claims); --first: with
              ModelConfig.first_claim (first-inserter claims, no settle passes).
  summarize:  python tools/shard_attr.py summarize TRACE_DIR R [--out f.json]
              reads rocprofv3's *_kernel_trace.csv (and *_memory_copy_trace.csv
              if present), keeps the last check (from the last R ClaimSet
              clears, one per rank at its init: the clear kernel or, on the
              compact table, a > 300 us fill), maps each Stream_Id to its rank
              by the order of those clears, and reports
              per rank the summed kernel time and the per-kernel split, the
              sum over ranks, the max over ranks (the critical path an R-GPU
              run would have, communication aside) and the check's span."""
import csv
import glob
import json
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(R, checks, tlc=False, first=False):
    sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))
    import torch  # noqa: F401  (owns the HIP runtime first)
    from kubecheck import ModelConfig
    from kubecheck.distributed import NativeShardedChecker
    mc = NativeShardedChecker(ModelConfig(np=2, keep_trace=False, tlc_order=tlc, first_claim=first), emulate=R)
    try:
        for k in range(checks):
            t0 = time.perf_counter()
            r = mc.run()
            dt = time.perf_counter() - t0
            print(json.dumps({"R": R, "check": k, "ms": round(dt * 1e3, 2), "distinct": r["distinct"],
                              "depth": r["depth"], "serial": os.environ.get("KC_SERIAL", "0"), "tlc": tlc,
                              "first": first, "claim_mode": r.get("claim_mode"),
                              "lib": os.path.basename(os.environ.get("KUBECHECK_LIB", "libkubecheck.so"))}),
                  flush=True)
    finally:
        mc.close()


def short(name):
    n = name.split("(")[0].replace("void ", "")
    for p in ("kc::", "hipcub::", "rocprim::detail::"):
        n = n.replace(p, "")
    return n.split("<")[0] if "<" in n and not n.startswith("k_claim") else n[:60]


def summarize(d, R, out):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(("k", r["Kernel_Name"], int(r["Stream_Id"]), int(r["Start_Timestamp"]),
                         int(r["End_Timestamp"])))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(("c", "copy " + r.get("Direction", "?"), int(r.get("Stream_Id", -1)),
                         int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort(key=lambda x: x[3])
    # every rank's check starts with its ClaimSet clear: the k_claimset_clear
    # kernel, or on the compact table of the first-claim mode a
    # hipMemsetAsync fill (the only fill of a warm check that runs > 300 us:
    # a rank's share of the table)
    clears = [i for i, r in enumerate(rows)
              if "k_claimset_clear" in r[1] or ("fillBuffer" in r[1] and r[4] - r[3] > 300_000)]
    if len(clears) < R:
        raise SystemExit(f"found {len(clears)} ClaimSet clears, need >= {R}")
    start = clears[-R]
    rank_of = {}
    for i in clears[-R:]:
        rank_of.setdefault(rows[i][2], len(rank_of))
    last = rows[start:]
    per = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    for kind, name, sid, t0, t1 in last:
        rk = rank_of.get(sid, -1)
        nm = short(name) if kind == "k" else name
        per[rk][nm] += (t1 - t0) / 1e6
        calls[rk][nm] += 1
    # per counted level (a level starts at its k_head_reset) of every rank:
    # kernel time and k_claim's share; narrow batches (k_sn_*) apart
    lv = defaultdict(list)
    for kind, name, sid, t0, t1 in last:
        rk = rank_of.get(sid, -1)
        if rk < 0 or kind != "k":
            continue
        nm = short(name)
        if nm.startswith("k_sn_"):
            continue
        if nm == "k_head_reset" or not lv[rk]:
            lv[rk].append([0.0, 0.0, 0])
        cur = lv[rk][-1]
        cur[0] += (t1 - t0) / 1e3
        cur[2] += 1
        if nm.startswith("k_claim"):
            cur[1] += (t1 - t0) / 1e3
    tot = {rk: sum(v.values()) for rk, v in per.items()}
    names = sorted({n for v in per.values() for n in v}, key=lambda n: -sum(per[r][n] for r in per))
    res = {"R": R, "span_ms": round((max(r[4] for r in last) - last[0][3]) / 1e6, 3),
           "sum_over_ranks_ms": round(sum(v for k, v in tot.items() if k >= 0), 3),
           "max_rank_ms": round(max((v for k, v in tot.items() if k >= 0), default=0), 3),
           "unattributed_ms": round(tot.get(-1, 0.0), 3),
           "per_rank_ms": {str(k): round(v, 3) for k, v in sorted(tot.items())},
           "per_kernel_ms": {n: {"sum": round(sum(per[r][n] for r in per), 3),
                                 "max_rank": round(max(per[r][n] for r in per if r >= 0) if any(r >= 0 for r in per) else 0, 3),
                                 "calls": sum(calls[r][n] for r in calls)} for n in names},
           # [kernel us, k_claim us, launches] per counted level, per rank
           "levels_us": {str(k): [[round(a, 1), round(b, 1), c] for a, b, c in v] for k, v in sorted(lv.items())}}
    print(json.dumps({k: v for k, v in res.items() if k != "levels_us"}, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    a = sys.argv[1:]
    if a and a[0] == "run":
        run(int(a[1]), int(a[a.index("--checks") + 1]) if "--checks" in a else 2, "--tlc" in a, "--first" in a)
    elif a and a[0] == "summarize":
        summarize(a[1], int(a[2]), a[a.index("--out") + 1] if "--out" in a else None)
    else:
        print(__doc__)
        sys.exit(2)
