"""Where a bench step's time goes outside the engine (diagnostic): per NP=2
check, the wall time of ModelChecker.run() against the engine's own clock
(kc_result.seconds, Init to finish), with and without the bench's HIP events
(timing=2: events around k_claim only) and with the bench's per-step
kernel_times()/narrow_times() calls.

  python3 tools/run_overhead.py [checks = 6]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

import kubecheck  # noqa: E402


def main(n: int) -> None:
    for timing in (0, 2):
        mc = kubecheck.ModelChecker(kubecheck.ModelConfig(np=2, keep_trace=True, timing=timing, fpset_slots=1 << 20,
                                                          first_claim=True))
        mc.run()
        walls, engs, calls = [], [], []
        for _ in range(n):
            t0 = time.perf_counter()
            r = mc.run()
            t1 = time.perf_counter()
            if timing:
                mc.kernel_times()
                mc.narrow_times()
            t2 = time.perf_counter()
            walls.append((t1 - t0) * 1e3)
            engs.append(r.seconds * 1e3)
            calls.append((t2 - t1) * 1e3)
        mc.close()
        print(json.dumps({"timing": timing, "run_wall_ms": [round(x, 3) for x in walls],
                          "engine_ms": [round(x, 3) for x in engs],
                          "outside_engine_ms": [round(a - b, 3) for a, b in zip(walls, engs)],
                          "kernel_times_calls_ms": [round(x, 3) for x in calls]}))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 6)
