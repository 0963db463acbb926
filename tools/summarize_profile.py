#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/:
  TAG_kernel_stats.csv   rocprofv3 --stats output (per-kernel calls / avg ns) of the bench --trace run
  TAG_traffic.json       per-frame kernel time and HBM bytes of the timed (non-counting) kernels:
                         kernel time = sum of their durations / the run's frames (warmup + timed),
                         checked against the bench line's kernel_ms; HBM bytes = 2 x FETCH_SIZE +
                         WRITE_SIZE (MI355X_MICROARCH.md §HBM: FETCH_SIZE tallies 128-B requests at
                         64 B on gfx950) summed the same way
  TAG_bench.jsonl        the bench JSON lines of the same build (--trace line, then the full line)
Also writes profiles/traffic_{batched,one_frame}.json (the files bench.py reads for `roofline.hbm`, by the
line's mode).
Counting-pass kernels (k_*<true>) are excluded; the untemplated kernels they share (k_pack_*, k_finish)
are charged their counting-pass calls at the average duration.

  python tools/summarize_profile.py TAG gpurun_out/prof_TAG
"""
import collections
import csv
import glob
import json
import re
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
tag, out = sys.argv[1], Path(sys.argv[2])
prof = ROOT / "profiles"
prof.mkdir(exist_ok=True)


def kname(s):
    """k_name, with '<true>' kept for counting-pass instantiations (k_finish's template argument is not
    COUNT but whether the launch's records are compact: both are the production kernel)."""
    m = re.search(r"(k_[a-z_0-9]+)(<(true|false)[,>])?", s)      # the first template argument: COUNT
    if not m:
        return s[:40]
    if m.group(1) in ("k_finish", "k_finish_any"):
        return m.group(1)
    return m.group(1) + ("<true>" if m.group(3) == "true" else "")


def lines(path):
    return [json.loads(l) for l in open(path) if l.startswith("{")] if path.exists() else []


trace = (lines(out / "trace.jsonl") or [{}])[-1]
full = (lines(out / "bench.jsonl") or [{}])[-1]
frame_kernels = trace.get("roofline", {}).get("kernels", [])
frames = trace.get("config", {}).get("trace_frames")
if not frames:
    sys.exit("trace.jsonl lacks config.trace_frames (run bench.py --trace)")

# kernel time per frame
stats = glob.glob(str(out / "kt" / "**" / "*kernel_stats.csv"), recursive=True)
per_kernel_ms, counting_calls = {}, 0
if stats:
    shutil.copy(stats[0], prof / f"{tag}_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats[0])))
    counting_calls = sum(int(r["Calls"]) for r in rows if kname(r["Name"]) == "k_chain<true>")
    agg = collections.defaultdict(lambda: [0, 0.0])              # calls, total ns (instantiations merged)
    for r in rows:
        k = kname(r["Name"])
        if k in frame_kernels:
            agg[k][0] += int(r["Calls"])
            agg[k][1] += float(r["TotalDurationNs"])
    for k, (calls, tot) in agg.items():
        if k in ("k_pack_a", "k_pack_b", "k_finish", "k_finish_any", "k_occlude", "k_fallback") and calls:
            tot -= min(calls, counting_calls) * tot / calls              # the counting passes' launches
        per_kernel_ms[k] = tot / frames / 1e6
kernel_ms_sum = sum(per_kernel_ms.values())

# HBM bytes per frame
per = collections.defaultdict(lambda: collections.defaultdict(list))
for pas in ("fetch", "write"):
    for f in glob.glob(str(out / pas / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
hbm = 0.0
per_kernel_bytes = {}
for k in frame_kernels:
    if k in per:
        b = (2.0 * sum(per[k].get("FETCH_SIZE", [])) + sum(per[k].get("WRITE_SIZE", []))) * 1024.0
        per_kernel_bytes[k] = b / frames
        hbm += b
hbm /= frames
# each kernel's ALGORITHMIC bytes per frame (the line's counting pass, bench.py kernel_bytes) beside its
# rocprof time and HBM bytes, so every per-kernel fraction can be recomputed from this file
rl = trace.get("roofline", {})
kb = dict(rl.get("alg_bytes_per_kernel") or {})
if kb:
    kb["k_occlude"] = kb.pop("k_occlude_a", 0) + kb.pop("k_occlude_b", 0)
peak = (rl.get("peak_measured") or {}).get("l2_line_gbps")
per_kernel_roofline = {}
for k, b in kb.items():
    t = per_kernel_ms.get(k)
    gbps = b / (t / 1e3) / 1e9 if t else None
    per_kernel_roofline[k] = {"alg_bytes_per_frame": b, "ms_per_frame_rocprof": t,
                              "achieved_gbps": round(gbps, 1) if gbps else None,
                              "frac_of_l2_line_peak": round(gbps / peak, 4) if gbps and peak else None,
                              "hbm_bytes_per_frame": per_kernel_bytes.get(k)}
mode = "batched" if (trace.get("config", {}).get("frames_in_flight") or 1) > 1 else "one_frame"
res = {"tag": tag, "mode": mode, "config": trace.get("config", {}).get("workload"), "aa": trace.get("config", {}).get("aa", 1),
       "path": trace.get("roofline", {}).get("path"),
       "frames": frames, "workspace_slots": trace.get("config", {}).get("workspace_slots"),
       "frames_in_flight": trace.get("config", {}).get("frames_in_flight"),
       "kernel_ms_per_frame_rocprof": kernel_ms_sum, "per_kernel_ms_per_frame": per_kernel_ms,
       "kernel_ms_bench_trace": trace.get("roofline", {}).get("kernel_ms"),
       "hbm_bytes_per_frame": hbm, "per_kernel_hbm_bytes_per_frame": per_kernel_bytes,
       "alg_bytes_per_frame": sum(kb.values()) if kb else None,
       "l2_line_peak_gbps": peak, "per_kernel_roofline": per_kernel_roofline,
       "note": "timed (non-counting) kernels only; per frame = run totals / (warmup + timed frames); "
               "HBM bytes = 2*FETCH_SIZE + WRITE_SIZE; alg bytes = the traced line's roofline.alg_bytes_per_kernel "
               "(k_occlude = A's + B's shadow walks); achieved = alg bytes / rocprof ms"}
(prof / f"{tag}_traffic.json").write_text(json.dumps(res, indent=1))
(prof / (f"traffic_{mode}.json" if res["aa"] == 1 else f"traffic_{mode}_aa{res['aa']}.json")).write_text(json.dumps(res, indent=1))
with open(prof / f"{tag}_bench.jsonl", "w") as f:
    for l in (trace, full):
        if l:
            f.write(json.dumps(l) + "\n")
print(json.dumps({k: res[k] for k in ("kernel_ms_per_frame_rocprof", "kernel_ms_bench_trace", "hbm_bytes_per_frame")}))
