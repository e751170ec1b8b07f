"""Time-to-counterexample with the deferred frontier:
NP=2 with the seeded resourceVersion race (variant 1, NoLostUpdate) fails
among a deferred level's rebuilt states: reported directly (engine.hip
report_deferred_invariant), or with KC_DEFER_DIRECT=0 redone from the
previous level on the materialising path (redo_from).  Compared with a clean
check of the same model to the same depth (variant 0, max_levels = the
error's depth) and with the whole run on the materialising path
(KC_DEFER=0).

  python tools/redo_cost.py [--reps 3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import torch  # noqa: E402,F401

from kubecheck import ModelChecker, ModelConfig  # noqa: E402


def timed(kw, reps, env=None):
    saved = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        with ModelChecker(ModelConfig(**kw)) as mc:
            r = mc.run()                    # warm: table growth, allocations
            t0 = time.perf_counter()
            for _ in range(reps):
                r = mc.run()
            dt = (time.perf_counter() - t0) / reps
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return r, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    bug = dict(np=2, variant=1, invariants=7)
    r, t_bug = timed(bug, a.reps)
    assert r.error == "invariant" and r.error_invariant == "NoLostUpdate", (r.error, r.error_invariant)
    depth = r.error_level
    r_m, t_mat = timed(bug, a.reps, {"KC_DEFER": "0"})
    assert (r_m.error_level, r_m.trace_len) == (r.error_level, r.trace_len)
    assert [list(map(int, x)) for x in r_m.trace] == [list(map(int, x)) for x in r.trace]
    r_r, t_redo = timed(bug, a.reps, {"KC_DEFER_DIRECT": "0"})
    assert [list(map(int, x)) for x in r_r.trace] == [list(map(int, x)) for x in r.trace]
    _, t_clean = timed(dict(np=2, invariants=7, max_levels=depth), a.reps)
    out = {"error_level": depth, "trace_len": r.trace_len, "redo_level_direct": r.defer_redo_level,
           "redo_level_redo": r_r.defer_redo_level,
           "ms_deferred_direct": round(t_bug * 1e3, 2), "ms_deferred_with_redo": round(t_redo * 1e3, 2),
           "ms_materialising": round(t_mat * 1e3, 2), "ms_clean_to_depth": round(t_clean * 1e3, 2),
           "direct_over_clean": round(t_bug / t_clean, 3), "redo_over_clean": round(t_redo / t_clean, 3),
           "materialising_over_clean": round(t_mat / t_clean, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
