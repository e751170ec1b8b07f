#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel trace/stats and --pmc passes) into
one JSON file under profiles/.

  python tools/pmc_summary.py --trace DIR [--fetch DIR] [--write DIR] --out profiles/X.json

Per kernel (template arguments stripped): calls and total/average duration
from the kernel trace, and the HBM traffic from the PMC passes, corrected as
MI355X_MICROARCH.md §HBM prescribes:
  * FETCH_SIZE and WRITE_SIZE are in KiB (bytes = value * 1024);
  * on gfx950 FETCH_SIZE reports 1/2 of the bytes actually fetched
    (TCC_EA0_RDREQ x 64 B tallied for 128-B requests), so it is doubled;
  * WRITE_SIZE is taken as is.
The per-launch figures are averages over every dispatch of that kernel.
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
            e["hbm_read_bytes_per_launch"] = 2 * kib * 1024 / n       # gfx950: FETCH_SIZE x2
        if k in write:
            n, kib = write[k]
            e["write_size_kib_per_launch_raw"] = kib / n
            e["hbm_write_bytes_per_launch"] = kib * 1024 / n
        if "hbm_read_bytes_per_launch" in e and "hbm_write_bytes_per_launch" in e:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_per_launch"] + e["hbm_write_bytes_per_launch"]
            e["hbm_GBps"] = round(e["hbm_bytes_per_launch"] / (e["avg_us"] * 1e3), 2)
        kernels[k] = e
    out = {"command": a.command,
           "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md §HBM)",
           "kernels": kernels}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, e in list(kernels.items())[:14]:
        print(f"{k:34s} calls {e['calls']:6d} total {e['total_ms']:9.3f} ms avg {e['avg_us']:9.2f} us"
              + (f"  hbm {e['hbm_bytes_per_launch'] / 1e6:10.3f} MB/launch {e['hbm_GBps']:8.1f} GB/s"
                 if "hbm_bytes_per_launch" in e else ""))


if __name__ == "__main__":
    main()
