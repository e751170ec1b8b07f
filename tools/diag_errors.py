"""Error reports of the native sharded loop under each combination of
KC_SNARROW / KC_SDEFER / KC_STAGE, for the error configurations of
tests/golden/oracle_fixtures.json (a diagnostic: which switch changes which
report).  python tools/diag_errors.py [R ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))
import torch  # noqa: E402,F401

from kubecheck import ModelConfig  # noqa: E402
from kubecheck.distributed import NativeShardedChecker  # noqa: E402

fx = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_fixtures.json")))
CASES = [("nc2", dict(nc=2)), ("variant2", dict(variant=2)), ("variant3", dict(variant=3)), ("ns0", dict(ns=0)),
         ("variant4", dict(variant=4)), ("variant1_lost_update", dict(variant=1, invariants=7))]
Rs = [int(a) for a in sys.argv[1:]] or [2]
for R in Rs:
    for env in ({"KC_SNARROW": "1", "KC_SDEFER": "1"}, {"KC_SNARROW": "0", "KC_SDEFER": "0"},
                {"KC_SNARROW": "0", "KC_SDEFER": "1"}, {"KC_SNARROW": "0", "KC_SDEFER": "1", "KC_STAGE": "0"}):
        os.environ.update(env)
        for key, kw in CASES:
            mc = NativeShardedChecker(ModelConfig(**kw), emulate=R)
            try:
                r = mc.run()
            finally:
                mc.close()
            f = fx[key]
            print(json.dumps({"R": R, "env": env, "case": key, "error": r["error"], "level": r["error_level"],
                              "trace_len": r["trace_len"], "want_level": f["err_level"],
                              "widths_ok": r["level_width"] == f["level_width"][:len(r["level_width"])]}),
                  flush=True)
        for k in env:
            os.environ.pop(k, None)
