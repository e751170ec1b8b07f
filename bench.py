#!/usr/bin/env python3
"""bench.py — distinct states/sec of the KubeAPI BFS model check on MI355X.

One "step" = one complete BFS safety check (TLC's hot path: expand, fingerprint,
FPSet dedup, invariant checks, parent pointers, next frontier) of the
BASELINE.json configs[1] model: KubeAPI with enlarged constants — 1 client,
2 PVC controllers, 1 API server, both REQUESTS_CAN_* TRUE (build-authored
parameterisation of KubeAPI.tla:161,225,268).  The
inputs are the model's Init states, so the timed region starts from an empty
FPSet with nothing precomputed.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload np2|model1|np3_52|fpset] [--deterministic]

Claims (round 6): by default the first inserter of a state owns it — TLC
-workers N semantics, the configuration of the reference's own recorded run
(KubeAPI___Model_1.launch:33, 4 workers): the same distinct/generated counts,
depth, level widths and counterexample lengths (checked against the golden
fixtures on every run).  The single-GPU line also times the deterministic
mode (every state's first discoverer is TLC -workers 1's: claim stores and
settle passes) under "deterministic"; --deterministic makes that the line.

N>1 runs one process per GPU (torch.distributed.run; a plain `python bench.py
--gpus N` starts that launcher itself as a child process) with the state
space sharded by fingerprint owner and one RCCL all-to-all per BFS level
(kubecheck.distributed); rank 0 prints one JSON line.  Every run's counts
are checked against the committed golden fixtures (tests/golden/).
"""
from __future__ import annotations

import argparse
import json
import re
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tla-kubernetes_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

WORKLOADS = {
    # name: (ModelConfig kwargs, description)
    "np2": (dict(nc=1, np=2, ns=1), "KubeAPI enlarged: NC=1 clients, NP=2 PVC controllers, NS=1 server"),
    "model1": (dict(nc=1, np=1, ns=1), "KubeAPI toolbox Model_1 (MC.cfg)"),
    # a scaling-sized workload: NP=3 (KubeAPI.tla:225 parameterised) has ~2e11
    # states, beyond 8 x 288 GB; its first 52 BFS levels (TLC -depth 52) hold
    # 1.1e9, with levels ~150-200M wide, where per-level costs do not dominate
    "np3_52": (dict(nc=1, np=3, ns=1, max_levels=52),
               "KubeAPI enlarged: NC=1, NP=3 PVC controllers, NS=1; the first 52 BFS levels"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="np2", choices=list(WORKLOADS) + ["fpset"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="budget of the CPU baseline sample (oracle)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="no per-kernel HIP events")
    ap.add_argument("--all-kernel-timing", action="store_true",
                    help="HIP events on every kernel (default: on the roofline kernel k_claim only;"
                         " events on all five per-level launches cost the NP=2 check ~6 ms)")
    ap.add_argument("--chunk", type=int, default=0, help="parents per expansion chunk (0 = default)")
    ap.add_argument("--deterministic", action="store_true",
                    help="the line in the deterministic claim mode (the first discoverer of every state is TLC "
                         "-workers 1's: settle passes) instead of the default first-claim mode (TLC -workers N "
                         "semantics, as the reference's own run, KubeAPI___Model_1.launch:33)")
    ap.add_argument("--first-claim", action="store_true",
                    help="(the default since round 6; kept for old command lines)")
    ap.add_argument("--no-second-line", "--no-first-claim-line", dest="no_second_line", action="store_true",
                    help="skip the single-GPU line's measurement of the other claim mode")
    ap.add_argument("--frontier-hbm-mb", type=int, default=0,
                    help="frontier spill mode: keep the frontiers in a StateQueue with this HBM budget")
    ap.add_argument("--fp-count", type=float, default=1e10,
                    help="fpset workload: fingerprints inserted (and looked up) per step")
    ap.add_argument("--fp-load", type=float, default=0.5, choices=[0.5, 0.75],
                    help="fpset workload: table load after the inserts")
    ap.add_argument("--sharded", action="store_true",
                    help="use the sharded (multi-GPU) stages even at N=1 (started under torch.distributed.run)")
    ap.add_argument("--deterministic-shards", action="store_true",
                    help="N>1 / --sharded: (rank, parent)-ordered minimum claims with their settle passes instead of "
                         "the sharded loop's default first-claim mode")
    ap.add_argument("--launcher-check", action="store_true",
                    help="only start the ranks (gloo, no GPU) and report what each saw: a CPU test of "
                         "the --gpus N self-launch")
    return ap.parse_args()


def launcher_check(args) -> dict:
    """Every rank joins a gloo group and all-gathers (rank, world, local rank)."""
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    mine = torch.tensor([rank, world, int(os.environ.get("LOCAL_RANK", "-1"))], dtype=torch.int64)
    out = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(out, mine)
    dist.destroy_process_group()
    if rank != 0:
        return None
    return {"launcher_check": True, "n_gpus": args.gpus, "world": world,
            "ranks": [o.tolist() for o in out],
            "master_addr": os.environ.get("MASTER_ADDR")}


def state_bytes(kw) -> int:
    import kubecheck

    return 8 * kubecheck.Spec(kubecheck.ModelConfig(**kw)).state_words


def roofline_bfs(times, res, S):
    """Roofline of the dominant kernel from HIP-event times over the timed steps.

    Algorithmic bytes per unit:
      claim  (k_claim)      : per parent S (frontier read); per GENERATED
                              successor 64 (one 64-B probe line, SURVEY's FPSet
                              op).  The kernel's LDS tile dedup lets about half
                              of the successors skip their probe, so the
                              achieved figure is an effective rate; `traffic`
                              (PMC) is what the kernel actually moved.  A
                              parent of a deferred frontier is
                              rebuilt there: + S (its state written into the
                              frontier) + 9 (its trace entry read) + 8 (its
                              parent's successor plan read); the read of its
                              own parent is the S above; and every parent's
                              plan is written for the next level (+ 8).
      settle (k_settle_rec) : per candidate 12 (record read) + 64 (probe line);
                              per parent 8 (newmask + newcnt write)
      emit   (k_emit)       : per parent 8 (mask + offset); per new state S + 9
                              (frontier write + parent pointer + ordinal) + S
                              (parent state re-read)
      scan                  : per parent 8
    """
    parents = res["parents"]
    dfr = res.get("deferred", 0)
    per_kernel = {
        "expand": parents * S + res["succ"] * 64 + (dfr * (S + 17) + parents * 8 if dfr else 0),
        "resolve": res["settles"] * (12 + 64) + parents * 8,
        # (deferred levels: k_emit_links writes only the 9-B trace entry)
        "emit": parents * 8 + res["new"] * (2 * S + 9) if not dfr else parents * 8 + res["new"] * 9,
        "scan": parents * 8,
        # k_narrow runs whole levels (expand + probe + emit); its bytes are
        # only attributable when it ran every level of the check
        "narrow": parents * S + res["succ"] * 64 + res["new"] * (2 * S + 9),
    }
    kernel_names = {"expand": "k_claim", "resolve": "k_settle_rec", "emit": "k_emit",
                    "scan": "rocprim scan", "narrow": "k_narrow"}
    name = max(times, key=lambda k: times[k][0])
    ms, launches = times[name]
    byts = per_kernel[name]
    achieved = byts / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    return name, {
        "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
        "kernel": kernel_names[name], "launches": launches,
        "avg_launch_us": round(ms * 1e3 / max(launches, 1), 2),
        "bytes_per_launch": int(byts / max(launches, 1)),
    }


def claim_ceiling():
    """The newest committed mixed-operation ceiling of k_claim's claim protocol
    (tools/microbench/claim_ceiling.hip -> profiles/<round>_claim_ceiling.json)."""
    import glob

    def run_order(f):
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, os.path.basename(f))

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_claim_ceiling.json")), key=run_order, reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
            d["ceiling_ms"]["deterministic"], d["per_check"]["claims"]
            return d, os.path.relpath(f, ROOT)
        except (OSError, ValueError, KeyError):
            continue
    return None, None


def claimset_compact(first: bool) -> bool:
    """The engine's first-claim ClaimSet holds 8-B fp words (round 6,
    DevClaimSet::compact) unless KC_CLAIM_COMPACT=0."""
    return first and os.environ.get("KC_CLAIM_COMPACT", "1") != "0"


def op_rate_roofline(kclaim_ms: float, probes: int, inserts: int, checks: int, first: bool) -> dict:
    """The roofline that bounds k_claim: its random memory
    OPERATIONS — per check every ClaimSet claim is one first-slot 16-B load,
    every new state one inserting CAS and, in the deterministic protocol, one
    agent-scope claim store — measured TOGETHER, in k_claim's own ratio and
    with the product's claimset_* code on a 2^32-slot (64 GiB) table like the
    NP=2 ClaimSet, by tools/microbench/claim_ceiling.hip with nothing else
    running (profiles/*_claim_ceiling.json).  ceiling_ms = that time scaled
    to this run's claims; frac = ceiling_ms / k_claim's time (<= 1: the share
    of the kernel's time its claims would need at the memory system's mixed
    random-operation rate; 1 - frac is what overlapping them with the
    successor computation has not hidden).  The per-kind fractions use the
    same table's isolated rates."""
    cal, src = claim_ceiling()
    t = kclaim_ms * 1e-3
    out = {"bound": "random-op rate (mixed, measured)", "kernel": "k_claim", "kernel_ms": round(kclaim_ms, 3),
           "claims": "first inserter" if first else "deterministic (claim store)",
           "probes": int(probes), "probes_per_s": round(probes / t, 1) if t else 0.0,
           "cas": int(inserts), "cas_per_s": round(inserts / t, 1) if t else 0.0,
           "claim_stores": 0 if first else int(inserts)}
    if cal is None or not t:
        out["frac"] = None
        out["source"] = "no committed claim-ceiling profile"
        return out
    mode = "first" if first else "deterministic"
    if claimset_compact(first) and "first_compact" in cal["ceiling_ms"]:
        mode = "first_compact"      # (the same claims on the compact table the engine uses)
    per_check = cal["ceiling_ms"][mode]
    ceil_ms = per_check * (probes / max(checks, 1)) / cal["per_check"]["claims"] * checks
    iso = cal["isolated_64GiB_G_per_s"]
    out.update({
        "ceiling_ms": round(ceil_ms, 3), "frac": round(ceil_ms / kclaim_ms, 4),
        "ceiling_claims_per_s": round(cal["per_check"]["claims"] / (per_check * 1e-3), 1),
        "probe_frac_isolated": round(probes / t / (iso["first_slot_load16"] * 1e9), 4),
        "cas_frac_isolated": round(inserts / t / (iso["cas_insert"] * 1e9), 4),
        "store_frac_isolated": 0.0 if first else round(inserts / t / (iso["agent_store8"] * 1e9), 4),
        "source": f"{src}: {mode} claims at {per_check} ms per NP=2 check ({cal['per_check']['claims']} claims, "
                  f"{cal['per_check']['units_new_states']} inserts), scaled by this run's claims per check; "
                  "isolated rates on the same 64 GiB table"})
    return out


def pmc_traffic(workload: str, kernel: str, stream_read_bytes: float = 0.0):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3
    summary for this workload (profiles/<round>_<workload>_rocprof_summary.json,
    written by tools/pmc_summary.py from separate FETCH_SIZE / WRITE_SIZE
    passes).  Corrected with our calibration (profiles/r02b_pmc_calibration.json):
    the random probes are reported at full size, the kernel's coalesced
    streaming reads (`stream_read_bytes` per launch, algorithmic) at half,
    writes as the interface carries them.  bench.py cannot collect PMC
    counters itself (they need their own rocprofv3 run), so the figure is
    the profile's."""
    import glob

    def run_order(f):      # r03z < r03aa < r03an: round, then tag length, then tag
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, os.path.basename(f))

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{workload}_rocprof_summary.json")), key=run_order)
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
            k = d["kernels"].get(kernel, {})
        except (OSError, ValueError, KeyError):
            continue
        if "fetch_bytes_per_launch_raw" in k and "write_bytes_per_launch_raw" in k:
            b = k["fetch_bytes_per_launch_raw"] + stream_read_bytes / 2 + k["write_bytes_per_launch_raw"]
            return int(b), os.path.relpath(f, ROOT), d.get("build_id")
    return None, None, None


def set_traffic(roof: dict, traffic, src, bid) -> None:
    """roofline.traffic is a PMC measurement only when the committed profile
    was taken on the kernels of this build (same kubecheck.build_id); an
    older profile's figure goes to traffic_estimate, traffic stays null."""
    from kubecheck._lib import build_id

    if traffic is None:
        return
    if bid == build_id():
        roof["traffic"] = traffic
        roof["traffic_unit"] = "HBM bytes per launch (PMC)"
        roof["traffic_source"] = f"{src} (build {bid}, this build)"
    else:
        roof["traffic"] = None
        roof["traffic_estimate"] = traffic
        roof["traffic_source"] = (f"{src}: PMC of build {bid or 'unrecorded'}, not this build "
                                  f"({build_id()}); an estimate, not a measurement of these kernels")


def host_cpu_info() -> dict:
    """The host CPUs the comparator may use: this process's affinity set, the
    machine's count, and the per-GPU share the GPU box grants (its
    OMP_NUM_THREADS, 16: os.cpu_count() there shows the whole host, whose
    other CPUs belong to the other GPUs' jobs)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16
    return {"affinity_cpus": aff, "machine_cpus": os.cpu_count() or aff, "per_gpu_share": share,
            "threads": max(1, min(share, aff))}


def host_cores() -> int:
    """Threads for the CPU comparator: this process's CPUs, capped at the
    box's per-GPU CPU share (host_cpu_info)."""
    return host_cpu_info()["threads"]


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(kw, seconds):
    """The CPU comparator (TLC's -workers = all host cores role):
    the oracle's multi-threaded BFS of the same model from Init, on this
    process's host cores (<= 16), stopped after `seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    info = host_cpu_info()
    threads = info["threads"]
    cfg = pyoracle.config(kw["nc"], kw["np"], kw["ns"], keep_trace=False)
    cfg.fpset_log2 = 22 if (kw["nc"], kw["np"], kw["ns"]) == (1, 1, 1) else 29
    r = pyoracle.bench_parallel(cfg, threads, seconds)
    what = "the whole model" if r["complete"] else f"{r['levels']} BFS levels from Init"
    out = {"value": round(r["rate"], 1), "unit": "distinct states/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(), "host_cpus": info,
           "cores_note": f"{threads} threads = min(this process's {info['affinity_cpus']} affinity CPUs, the box's "
                         f"per-GPU CPU share {info['per_gpu_share']}); the machine has {info['machine_cpus']}",
           "sample": f"oracle/kubeapi_oracle.c ko_bench_parallel: level-synchronous BFS of the same "
                     f"model on {threads} threads with a lock-free 64-bit fingerprint set, {what} "
                     f"({r['distinct']} distinct, {r['generated']} generated) in {r['seconds']:.1f} s"}
    # the same comparator over the WHOLE model, run once on a GPU box's host
    # (tools/gpu_prof_r02.sh ... cpu): too long for every bench run
    if (kw["nc"], kw["np"], kw["ns"]) == (1, 2, 1):
        import glob
        # the whole model at 16, 64, 128 and all 256 affinity CPUs of a GPU
        # box's host (tools/gpu.sh probe): the box's CPU share makes more
        # threads slower, so 16 is the comparator's best
        sweep = []
        for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r04a_cpu_np2_full_t*.json"))):
            try:
                with open(f) as fh:
                    full = json.load(fh)
                sweep.append({"threads": full["threads"], "seconds": full["seconds"],
                              "distinct_per_s": full["distinct_per_s"], "exact": full["distinct"] == 740607995,
                              "source": os.path.relpath(f, ROOT)})
            except (OSError, ValueError, KeyError):
                pass
        if sweep:
            sweep.sort(key=lambda e: e["threads"])
            best = max(sweep, key=lambda e: e["distinct_per_s"])
            out["full_model_run"] = dict(best)
            out["full_model_thread_sweep"] = sweep
    return out


def bench_single(args, kw, desc):
    import torch
    import kubecheck

    cfg = kubecheck.ModelConfig(**kw, keep_trace=True,
                                timing=0 if args.no_timing else (1 if args.all_kernel_timing else 2),
                                fpset_slots=1 << 20, chunk_states=args.chunk,
                                frontier_hbm_bytes=args.frontier_hbm_mb << 20, first_claim=not args.deterministic)
    mc = kubecheck.ModelChecker(cfg)
    cold_ms = None
    for w in range(args.warmup):
        tw = time.perf_counter()
        mc.run()
        torch.cuda.synchronize()
        if w == 0:        # a fresh engine: the ClaimSet grows by rehash from 2^20 slots
            cold_ms = round((time.perf_counter() - tw) * 1e3, 3)
    torch.cuda.synchronize()
    times = {"expand": [0.0, 0], "resolve": [0.0, 0], "scan": [0.0, 0], "emit": [0.0, 0]}
    acc = {"parents": 0, "probes": 0, "succ": 0, "new": 0, "settles": 0, "deferred": 0}
    narrow = [0.0, 0, 0]          # narrow-level kernel: ms, launches, levels
    t0 = time.perf_counter()
    results = []
    for _ in range(args.steps):
        r = mc.run()
        results.append(r)
        kt = mc.kernel_times()
        for k in times:
            times[k][0] += kt[k][0]
            times[k][1] += kt[k][1]
        nt = mc.narrow_times()
        narrow = [narrow[0] + nt[0], narrow[1] + nt[1], narrow[2] + nt[2]]
        acc["parents"] += r.distinct - r.queue_left
        acc["probes"] += r.fpset_probes
        acc["settles"] += r.batch_inserts
        acc["succ"] += r.generated - r.init
        acc["new"] += r.distinct - r.init
        acc["deferred"] += r.deferred_states
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    r = results[-1]
    assert all((x.distinct, x.generated) == (r.distinct, r.generated) for x in results)
    assert (r.complete or kw.get("max_levels")) and r.error is None
    golden = golden_check(args.workload, {"distinct": r.distinct, "generated": r.generated,
                                          "depth": r.depth, "level_width": r.level_width})
    out = {
        "metric": "distinct states/sec (KubeAPI TLC BFS)",
        "value": round(r.distinct * args.steps / dt, 1),
        "unit": "distinct states/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u64", "data": "synthetic (the model's Init states; no external input)",
        "config": {"workload": desc, "model": f"nc={kw['nc']},np={kw['np']},ns={kw['ns']}"
                   + (f",max_levels={kw['max_levels']}" if kw.get("max_levels") else ""),
                   "constants": "REQUESTS_CAN_FAIL=TRUE,REQUESTS_CAN_TIMEOUT=TRUE",
                   "invariants": "TypeOK,OnlyOneVersion", "distinct": r.distinct,
                   "generated": r.generated, "depth": r.depth, "parallelism": "1 GPU",
                   "path": "single-GPU engine (kc_engine_run)" + (
                       f", frontiers in the StateQueue with a {args.frontier_hbm_mb} MiB HBM budget"
                       if args.frontier_hbm_mb else ""), "golden_check": golden,
                   "claimset_probes": r.fpset_probes, "settle_reads": r.batch_inserts,
                   "chunks": r.levels_chunks, "deferred_frontier_states": r.deferred_states,
                   "deferred_frontier_redone": r.defer_fallback, "narrow_levels": r.narrow_levels,
                   "cold_first_check_ms": cold_ms,
                   # (the mode the engine reports it ran, kc_result.claim_mode: a flag the engine
                   # cannot honour, e.g. with a frontier HBM budget, does not relabel the line)
                   "claims": ("first inserter (TLC -workers N semantics: same counts and trace lengths; "
                              "the winning copy of a same-level duplicate is not deterministic)"
                              if r.claim_mode == "first" else "sequential-BFS minimum (TLC -workers 1 order)"),
                   "claim_mode": r.claim_mode,
                   "claimset": f"{r.fpset_slots} slots x {8 if claimset_compact(r.claim_mode == 'first') else 16} B",
                   "cold_first_check_note": "the first (warmup) check of a fresh engine, its ClaimSet grown by "
                                            "rehash from 2^20 slots; the timed checks reuse the grown table "
                                            "(cleared each check), like TLC's -fpmem pre-sizing"},
    }
    if not args.no_timing:
        S = state_bytes(kw)
        tt = {k: tuple(v) for k, v in times.items()}
        if narrow[1] and narrow[2] // args.steps >= r.depth - 1:     # every level ran narrow
            tt["narrow"] = (narrow[0], narrow[1])
        name, roof = roofline_bfs(tt, acc, S)
        # k_claim streams its parents (S B each); everything else it reads is a random probe
        stream = acc["parents"] * S / max(times["expand"][1], 1) if roof["kernel"] == "k_claim" else 0.0
        set_traffic(roof, *pmc_traffic(args.workload, roof["kernel"], stream))
        if roof["kernel"] == "k_claim":
            roof["op_rate"] = op_rate_roofline(times["expand"][0], acc["probes"], acc["new"], args.steps,
                                               r.claim_mode == "first")
        out["roofline"] = roof
        out["kernel_ms_per_step"] = {k: round(v[0] / args.steps, 3) for k, v in times.items() if v[0] > 0}
        if narrow[1]:
            out["kernel_ms_per_step"]["narrow"] = round(narrow[0] / args.steps, 3)
            out["config"]["narrow_levels_per_step"] = narrow[2] // args.steps
    mc.close()
    if not args.no_second_line and not args.frontier_hbm_mb:
        # the other claim mode, timed the same way (the headline in
        # first-claim mode only with the deterministic figure beside it)
        out["deterministic" if r.claim_mode == "first" else "first_claim"] = other_mode_line(args, cfg, r)
    return out


def other_mode_line(args, cfg, ref):
    """The same check in the other claim mode (ModelConfig.first_claim flipped),
    timed the same way beside the headline, with its own k_claim time and
    op-rate fraction: counts, depth and every level width must equal the
    headline run's (the claim mode decides only which same-level copy of a
    state is its first discoverer)."""
    import dataclasses
    import torch
    import kubecheck

    first = not cfg.first_claim
    mc = kubecheck.ModelChecker(dataclasses.replace(cfg, first_claim=first, timing=0 if args.no_timing else 2))
    for _ in range(args.warmup):
        mc.run()
    torch.cuda.synchronize()
    kms, probes, new = 0.0, 0, 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = mc.run()
        if (r.distinct, r.generated, r.depth, r.level_width) != (ref.distinct, ref.generated, ref.depth,
                                                                  ref.level_width):
            raise RuntimeError("bench: the other claim mode changed the counts")
        kms += mc.kernel_times()["expand"][0]
        probes += r.fpset_probes
        new += r.distinct - r.init
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    mc.close()
    out = {"value": round(r.distinct * args.steps / dt, 1), "ms_per_step": round(dt * 1e3 / args.steps, 3),
           "claim_mode": r.claim_mode, "defer_fallback": r.defer_fallback, "settle_reads": r.batch_inserts,
           "counts_equal_headline": True,
           "note": ("ModelConfig(first_claim=False): every state's first discoverer is the sequential-BFS "
                    "minimum (TLC -workers 1), at the cost of the claim stores and two settle passes"
                    if r.claim_mode == "minimum" else
                    "ModelConfig(first_claim=True): the first ClaimSet inserter owns a state, as in a TLC "
                    "-workers N run; no settle passes")}
    if kms > 0:
        out["k_claim_ms_per_step"] = round(kms / args.steps, 3)
        out["op_rate_frac"] = op_rate_roofline(kms, probes, new, args.steps, r.claim_mode == "first")["frac"]
    return out


def bench_fpset(args):
    """BASELINE config 4: insert fp_count device-generated fingerprints into a
    table sized for a final load of fp_load, then look up as many (half
    present, half absent).  One 64-B HBM burst per random probe is the
    algorithmic traffic of an insert (the 16-B pair it reads lives in it)."""
    import torch
    import kubecheck

    n = int(args.fp_count)
    batch = 1 << 24
    cap = int(n / args.fp_load * 3 / 4)   # kc_fpset_create sizes slots = 4/3 * capacity
    s = None
    for _ in range(args.warmup):
        if s is not None:
            s.close()
        s = kubecheck.FPSet(capacity=cap)
        s.stress(0x5EED0000, n, batch, n)   # perm63 stream (kc_fpset_stress)
    torch.cuda.synchronize()
    tin = tlk = 0.0
    for k in range(args.steps):
        if s is not None:
            s.close()
        s = kubecheck.FPSet(capacity=cap)
        ti, tl, found = s.stress(0x5EED0000 + k, n, batch, n)
        # the perm63 stream has no duplicates: every count is exact
        if s.size() != n or found != (n + 1) // 2:
            raise RuntimeError(f"fpset stress: size {s.size()} found {found} for {n} inserts")
        tin += ti
        tlk += tl
    load, table_bytes = s.size() / s.capacity(), s.capacity() * 8
    s.close()
    gbs = n * args.steps * 64 / tin / 1e9
    out = {
        "metric": "FPSet probe HBM GB/s (insert)", "value": round(gbs, 1), "unit": "GB/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(tin * 1e3 / args.steps, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic perm63 fingerprint stream generated on device",
        "config": {"workload": f"FPSet stress: {n} inserts + {n} lookups to {load:.0%} load, batch {batch}",
                   "table_bytes": table_bytes,
                   "inserts_per_s": round(n * args.steps / tin, 1),
                   "lookups_per_s": round(n * args.steps / tlk, 1),
                   "lookups_found": int(found)},
        "roofline": {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "k_stress_insert", "bytes_per_launch": batch * 64},
    }
    set_traffic(out["roofline"], *pmc_traffic("fpset", "k_stress_insert"))
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_fpset(args.fp_load)
    return out


def cpu_baseline_fpset(load: float) -> dict:
    """The FPSet stress on the host: the same
    open-addressing set shape in host RAM, filled by all the comparator's
    threads with lock-free CAS inserts (oracle/fpset_cpu.c), on a bounded
    sample of 2^28 fingerprints (a 4 GiB table at 50% load)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    info = host_cpu_info()
    n = 1 << 28
    r = pyoracle.fpset_stress_cpu(n, load, info["threads"])
    if r["inserted"] != n or r["found"] != n // 2:
        raise RuntimeError(f"fpset cpu comparator: {r}")
    return {"value": round(r["inserts_per_s"] * 64 / 1e9, 2), "unit": "GB/s", "cores": info["threads"],
            "kind": "port", "cpu_model": cpu_model(), "host_cpus": info,
            "inserts_per_s": round(r["inserts_per_s"], 1), "lookups_per_s": round(r["lookups_per_s"], 1),
            "sample": f"oracle/fpset_cpu.c: {n} distinct fingerprints inserted by {info['threads']} threads "
                      f"(lock-free CAS, linear probing) into a {r['slots'] * 8 >> 20} MiB host table to "
                      f"{load:.0%} load in {r['insert_seconds']:.2f} s, then {n} lookups (half present) in "
                      f"{r['lookup_seconds']:.2f} s; value = inserts/s x 64 B, the GPU line's unit"}


def relaunch(args) -> int:
    """`python bench.py --gpus N` (or `--sharded` at N=1) without a
    torch.distributed launcher: start
    N ranks under torch.distributed.run as a CHILD process (nothing here has
    touched the GPU; no exec) and return its exit code."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def golden_check(workload: str, res: dict) -> str:
    """Counts of a bench run against the committed fixtures: NP=2 against the
    oracle's full run (tests/golden/np2_full.json), Model_1 against MC.out
    (tests/golden/model1_mcout.json) and the oracle's level widths."""
    g = os.path.join(ROOT, "tests", "golden")
    if workload == "np2":
        fx = json.load(open(os.path.join(g, "np2_full.json")))
        want = (fx["distinct"], fx["generated"], fx["depth"], fx["level_width"])
        src = "tests/golden/np2_full.json"
    elif workload == "np3_52":
        fx = json.load(open(os.path.join(g, "np3_52levels.json")))
        want = (fx["distinct"], fx["generated"], fx["depth"], fx["level_width"])
        src = "tests/golden/np3_52levels.json"
    else:
        mc = json.load(open(os.path.join(g, "model1_mcout.json")))
        fx = json.load(open(os.path.join(g, "oracle_fixtures.json")))["model1"]
        want = (mc["distinct"], mc["generated"], mc["depth"], fx["level_width"])
        src = "tests/golden/model1_mcout.json (MC.out:1098,1101) + oracle level widths"
    got = (res["distinct"], res["generated"], res["depth"], list(res["level_width"]))
    if got != want:
        raise RuntimeError(f"bench {workload}: counts differ from {src}: "
                           f"got {got[:3]} want {want[:3]} (widths equal: {got[3] == want[3]})")
    return src


def _json_stdout():
    """The bench's one JSON line goes to the original stdout; everything else
    written to file descriptor 1 from here on (RCCL prints its version banner
    there at communicator init, in every rank) goes to stderr, so stdout
    carries exactly one line."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if (args.gpus > 1 or args.sharded) and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args))
    jout = _json_stdout()
    if args.gpus != world and world != 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.launcher_check:
        out = launcher_check(args)
        if out is not None:
            print(json.dumps(out), file=jout, flush=True)
        return
    if args.workload == "fpset":
        if args.gpus > 1 or args.sharded:
            from kubecheck.sharded_fpset import bench_sharded_fpset

            out = bench_sharded_fpset(args)
            if out is None:          # not rank 0
                return
        else:
            out = bench_fpset(args)
    else:
        kw, desc = WORKLOADS[args.workload]
        if args.gpus > 1 or args.sharded:
            from kubecheck import distributed

            out = distributed.bench_sharded(args, kw, desc, golden_check)
            if out is None:          # not rank 0
                return
        else:
            out = bench_single(args, kw, desc)
        if not args.no_cpu_baseline:
            # rank 0 only (the other ranks returned above), after every rank's
            # timed region; at N > 1 a shorter sample keeps the run within minutes
            secs = args.cpu_seconds if args.gpus == 1 else min(args.cpu_seconds, 10.0)
            out["cpu_baseline"] = cpu_baseline(kw, secs)
    print(json.dumps(out), file=jout, flush=True)


if __name__ == "__main__":
    main()
