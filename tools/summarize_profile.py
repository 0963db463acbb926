#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/:
  TAG_kernel_stats.csv   rocprofv3 --stats output (per-kernel calls / avg ns)
  TAG_traffic.json       per-kernel FETCH_SIZE / WRITE_SIZE means and the HBM
                         bytes per frame: sum over the frame's kernels of
                         2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md §HBM:
                         FETCH_SIZE tallies 128-B requests at 64 B on gfx950)
  TAG_bench.jsonl        the bench JSON line of the same build
Also writes profiles/traffic.json (the file bench.py reads for `roofline.traffic`).
"""
import csv
import collections
import glob
import json
import os
import re
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
tag, out = sys.argv[1], Path(sys.argv[2])
prof = ROOT / "profiles"
prof.mkdir(exist_ok=True)


def kname(s):
    m = re.search(r"(k_[a-z_0-9]+)", s)
    return m.group(1) if m else s[:40]


stats = glob.glob(str(out / "kt" / "**" / "*kernel_stats.csv"), recursive=True)
if stats:
    shutil.copy(stats[0], prof / f"{tag}_kernel_stats.csv")

per = collections.defaultdict(lambda: collections.defaultdict(list))
for pas in ("fetch", "write"):
    for f in glob.glob(str(out / pas / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
kern = {}
for k, d in per.items():
    kern[k] = {c: sum(v) / len(v) for c, v in d.items()}
bench = [json.loads(l) for l in open(out / "bench.jsonl") if l.startswith("{")]
line = bench[-1] if bench else {}
frame_kernels = line.get("roofline", {}).get("kernels", [])
tot = 0.0
nframes = line.get("config", {}).get("frames_rendered_total")
if nframes:
    # frame batches: launches cover different frame counts, so divide the run's totals by its frames
    for k in frame_kernels:
        if k in per:
            tot += (2.0 * sum(per[k].get("FETCH_SIZE", [])) + sum(per[k].get("WRITE_SIZE", []))) * 1024.0
    tot /= nframes
else:
    for k in frame_kernels:
        if k in kern:
            tot += (2.0 * kern[k].get("FETCH_SIZE", 0.0) + kern[k].get("WRITE_SIZE", 0.0)) * 1024.0
res = {"tag": tag, "config": line.get("config", {}).get("workload"), "path": line.get("roofline", {}).get("path"),
       "per_kernel_KiB": kern, "frame_kernels": frame_kernels, "hbm_bytes_per_frame": tot,
       "frames_rendered_total": nframes,
       "note": "2*FETCH_SIZE + WRITE_SIZE per kernel (KiB), summed over one frame's kernels"
               + (" (run totals / frames_rendered_total)" if nframes else "")}
(prof / f"{tag}_traffic.json").write_text(json.dumps(res, indent=1))
(prof / "traffic.json").write_text(json.dumps(res, indent=1))
shutil.copy(out / "bench.jsonl", prof / f"{tag}_bench.jsonl")
print(json.dumps({"hbm_bytes_per_frame": tot, "kernels": frame_kernels}))
