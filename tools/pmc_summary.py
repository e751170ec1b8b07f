#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel trace/stats and --pmc passes) into
one JSON file under profiles/.

  python tools/pmc_summary.py --trace DIR [--fetch DIR] [--write DIR] --out profiles/X.json

Per kernel (template arguments stripped): calls and total/average duration
from the kernel trace, and the HBM traffic from the PMC passes.  FETCH_SIZE
and WRITE_SIZE are in KiB (bytes = value * 1024).  The correction follows
our own calibration (profiles/r02b_pmc_calibration.json, made with
tools/microbench/pmc_calib.hip as MI355X_MICROARCH.md §HBM asks for
uncalibrated shapes):
  * coalesced 16 B/lane streaming reads are reported at 1/2 (the guide's
    figure; 128-B requests tallied at 64 B);
  * random 16-B / 8-B loads are reported at their full 64-B request size;
  * atomics and random stores are reported as 64-B (CAS) or 32-B (max,
    8-B stores) write requests, streaming stores exactly.
So the raw FETCH_SIZE is exact for the random-probe part of a kernel and
half of its streaming part: hbm_read = raw + streaming_read_bytes / 2, where
the streaming bytes come from the caller's algorithmic count (bench.py
pmc_traffic); `hbm_bytes_per_launch_raw` = FETCH + WRITE as reported.  The
per-launch figures are averages over every dispatch of that kernel.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*$", "", name.strip())          # drop the parameter list
    n = re.sub(r"<.*>", "", n)                        # drop template arguments
    n = n.replace("void ", "").strip()
    return n.split("::")[-1]


def rows(d: str, suffix: str):
    for f in sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)):
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def kernel_trace(d: str):
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows(d, "kernel_trace.csv"):
        k = short(r.get("Kernel_Name", ""))
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return agg


def counters(d: str, name: str):
    agg = defaultdict(lambda: [0, 0.0])
    if not d:
        return agg
    for r in rows(d, "counter_collection.csv"):
        if r.get("Counter_Name") != name:
            continue
        k = short(r.get("Kernel_Name", ""))
        agg[k][0] += 1
        agg[k][1] += float(r["Counter_Value"])
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out", required=True)
    ap.add_argument("--command", default="")
    ap.add_argument("--algorithmic", help="JSON with the profiled run's algorithmic bytes (tools/sharded_profile.py)")
    a = ap.parse_args()
    trace = kernel_trace(a.trace)
    fetch, write = counters(a.fetch, "FETCH_SIZE"), counters(a.write, "WRITE_SIZE")
    kernels = {}
    for k, (calls, total_ms) in sorted(trace.items(), key=lambda kv: -kv[1][1]):
        e = {"calls": calls, "total_ms": round(total_ms, 4),
             "avg_us": round(total_ms * 1e3 / max(calls, 1), 3)}
        if k in fetch:
            n, kib = fetch[k]
            e["fetch_size_kib_per_launch_raw"] = kib / n
            e["fetch_bytes_per_launch_raw"] = kib * 1024 / n
        if k in write:
            n, kib = write[k]
            e["write_size_kib_per_launch_raw"] = kib / n
            e["write_bytes_per_launch_raw"] = kib * 1024 / n
        if "fetch_bytes_per_launch_raw" in e and "write_bytes_per_launch_raw" in e:
            e["hbm_bytes_per_launch_raw"] = e["fetch_bytes_per_launch_raw"] + e["write_bytes_per_launch_raw"]
            e["hbm_GBps_raw"] = round(e["hbm_bytes_per_launch_raw"] / (e["avg_us"] * 1e3), 2)
        kernels[k] = e
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tla-kubernetes_amd"))
    from kubecheck._lib import build_id
    out = {"command": a.command, "build_id": build_id(),
           "correction": "raw bytes = FETCH_SIZE*1024 + WRITE_SIZE*1024; hbm_read = raw fetch + "
                         "streaming_read/2 (profiles/r02b_pmc_calibration.json)",
           "kernels": kernels}
    if a.algorithmic:
        out["algorithmic"] = json.load(open(a.algorithmic))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, e in list(kernels.items())[:14]:
        print(f"{k:34s} calls {e['calls']:6d} total {e['total_ms']:9.3f} ms avg {e['avg_us']:9.2f} us"
              + (f"  raw {e['hbm_bytes_per_launch_raw'] / 1e6:10.3f} MB/launch {e['hbm_GBps_raw']:8.1f} GB/s"
                 if "hbm_bytes_per_launch_raw" in e else ""))


if __name__ == "__main__":
    main()
