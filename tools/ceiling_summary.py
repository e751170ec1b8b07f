"""Summarise a tools/microbench/claim_ceiling run (its JSON lines) into the
profile bench.py reads (profiles/<round>_claim_ceiling.json; bench.py
claim_ceiling() takes the newest).

  python3 tools/ceiling_summary.py gpurun_out/<tag>/ceiling.log <tag> > profiles/<tag>_claim_ceiling.json
"""
import json
import sys


def main(log: str, tag: str) -> None:
    rows = [json.loads(l) for l in open(log) if l.startswith("{")]
    iso = next(r for r in rows if r.get("isolated"))
    summ = next(r for r in rows if r.get("summary"))
    runs = [r for r in rows if "mode" in r]
    ceil = {"deterministic": summ["deterministic_ms"], "first": summ["first_ms"]}
    best = {"deterministic": summ["deterministic_K"], "first": summ["first_K"]}
    if "first_compact_ms" in summ:
        ceil["first_compact"] = summ["first_compact_ms"]
        best["first_compact"] = summ["first_compact_K"]
    ns = summ["table_slots"]
    out = {
        "tool": "tools/microbench/claim_ceiling.hip (VERDICT r5 item 2): k_claim's claim-protocol memory "
                "operations alone, per NP=2 check, with the product's claimset_* code on a "
                f"{ns}-slot ClaimSet (16-B slots = {ns * 16 >> 30} GiB; first_compact: the first-claim "
                f"mode's compact table, 8-B fp words = {ns * 8 >> 30} GiB); one unit = one new fingerprint "
                "(first-slot load, CAS, and in the deterministic protocol the agent-scope claim store) + "
                "the run's lookups of fingerprints stored earlier (first-slot load, found)",
        "command": f"./tools/microbench/claim_ceiling (gpurun {tag})",
        "box": f"MI355X, gpurun {tag}",
        "per_check": {"units_new_states": summ["units"], "claims": summ["probes"], "prefill": summ["prefill"],
                      "table_slots": ns},
        "ceiling_ms": ceil,
        "best_K": best,
        "isolated_64GiB_G_per_s": {"first_slot_load16": iso["load_G_per_s"], "cas_insert": iso["cas_G_per_s"],
                                   "agent_store8": iso["store_G_per_s"]},
        "runs": len(runs),
        "run_lines": runs,
        "note": "K = units per lane with all their first-slot loads issued together; the fastest K is the ceiling.",
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
