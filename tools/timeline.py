#!/usr/bin/env python3
"""The last call of a rocprofv3 kernel trace (bench.py --trace: the timed frames come last, after a host
gap), as a per-stream timeline: each kernel's start/end relative to the call's first kernel, the time
with k kernels running, and per kernel name the summed duration and the union of its intervals.

  python tools/timeline.py gpurun_out/tl20/<host>/<pid>/run_kernel_trace.csv [--gap-ms 0.5]
"""
import argparse
import csv
import json
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            short = name.replace("void ", "").replace("rtc::", "").replace("(anonymous namespace)::", "")
            short = short.split("(")[0].strip()
            rows.append({"name": short, "s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"]),
                         "q": r.get("Stream_Id") or r.get("Queue_Id", "?")})
    rows.sort(key=lambda x: x["s"])
    return rows


def last_call(rows, gap_ns):
    end = rows[0]["e"]
    start_ix = 0
    for i, r in enumerate(rows[1:], 1):
        if r["s"] - end > gap_ns:
            start_ix = i
        end = max(end, r["e"])
    return rows[start_ix:]


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--gap-ms", type=float, default=0.5)
    ap.add_argument("--streams", action="store_true", help="print every stream's kernel sequence")
    ap.add_argument("--prefix", default="k_", help="only kernels whose short name starts with this ('' all)")
    a = ap.parse_args()
    rows = [r for r in load(a.csv) if r["name"].startswith(a.prefix)]
    call = last_call(rows, int(a.gap_ms * 1e6))
    t0 = call[0]["s"]
    t1 = max(r["e"] for r in call)
    ev = []
    for r in call:
        ev.append((r["s"], 1))
        ev.append((r["e"], -1))
    ev.sort()
    conc = defaultdict(int)
    k, last = 0, t0
    for t, d in ev:
        conc[k] += t - last
        k += d
        last = t
    per = defaultdict(lambda: {"n": 0, "sum_ms": 0.0, "iv": []})
    for r in call:
        p = per[r["name"]]
        p["n"] += 1
        p["sum_ms"] += (r["e"] - r["s"]) / 1e6
        p["iv"].append((r["s"], r["e"]))
    out = {"window_ms": round((t1 - t0) / 1e6, 4), "kernels": len(call),
           "ms_with_k_running": {str(k): round(v / 1e6, 4) for k, v in sorted(conc.items())},
           "per_kernel": {n: {"launches": p["n"], "sum_ms": round(p["sum_ms"], 4),
                              "union_ms": round(union(p["iv"]) / 1e6, 4),
                              "first_start_ms": round((min(s for s, _ in p["iv"]) - t0) / 1e6, 4),
                              "last_end_ms": round((max(e for _, e in p["iv"]) - t0) / 1e6, 4)}
                          for n, p in per.items()}}
    print(json.dumps(out, indent=1))
    if a.streams:
        bys = defaultdict(list)
        for r in call:
            bys[r["q"]].append(r)
        for q, rs in bys.items():
            print(f"stream {q}: " + "  ".join(f"{r['name']}[{(r['s'] - t0) / 1e6:.3f}-{(r['e'] - t0) / 1e6:.3f}]"
                                              for r in rs))


if __name__ == "__main__":
    main()
