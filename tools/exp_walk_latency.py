#!/usr/bin/env python3
"""Dependent-step latency of single closest-hit walks (rt_walk_timing).

The rays (tools/heavy_rays_c3.txt, hex floats: o.xyz dir.xyz) are the mirror
chain of the C3 frame's heaviest pixel (row 495, col 1227) followed by an
ordinary eye ray, dumped by tools/exp_sah_closest.cpp --dump.  One wave walks
each ray alone (1 lane) or with 64 lanes on the same ray, on the 4-wide tree
(mode 0), on the reference tree (mode 1), memory-only chases (modes 3, 4) and as a cooperative walk
(mode 5: coop_step, 8 lanes, one wide-node slot per lane); cycles are s_memtime ticks.
"""
import json
import sys
import tempfile
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as graft  # noqa: E402

pkg = graft.import_pkg()
rays = np.array([[float.fromhex(x) for x in l.split()] for l in
                 (Path(__file__).parent / "heavy_rays_c3.txt").read_text().splitlines() if l.strip()], dtype=np.float32)
xml = pkg.scenes.write_config("C3_hm_1080p_d6", tempfile.mkdtemp())
s = pkg.Scene.from_xml(xml, device=0)
res = {}
for mode in (0, 1, 3, 4, 5):
    for lanes in ((1, 8, 64) if mode < 2 else (8,)):
        o = s.walk_timing(rays, lanes=lanes, reps=4, mode=mode)
        res[f"mode{mode}_lanes{lanes}"] = [{"cycles": int(a), "steps": int(b), "prim": int(np.int64(c)), "cold": int(d),
                                            "cyc_per_step": round(int(a) / max(1, int(b)), 1)} for a, b, c, d in o]
print(json.dumps(res, indent=1))
