#!/usr/bin/env python3
"""Experiment: is the frame time bound by the critical path (slowest pixel chain)?

Times (a) crops of the C3 frame around its heaviest pixels (row ~505, col ~1310,
found with oracle work maps) and (b) the full frame at MaxRecursionDepth 0..6,
for both render paths.  Crops are re-projected cameras (narrower near plane),
so rays differ in the last ulp from the full frame; only timing matters here.
"""
import json
import os
import sys
import tempfile
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as graft  # noqa: E402

pkg = graft.import_pkg()
d = tempfile.mkdtemp()
xml = pkg.scenes.write_config("C3_hm_1080p_d6", d)
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)


def crop(cam, r0, c0, h, w):
    c = pkg.Camera()
    c.position, c.gaze, c.up = cam.position, cam.gaze, cam.up
    l, r, b, t = cam.near_plane
    W, H = cam.image_width, cam.image_height
    su, sv = (r - l) / W, (t - b) / H
    c.near_plane[0] = l + su * c0
    c.near_plane[1] = l + su * (c0 + w)
    c.near_plane[3] = t - sv * r0
    c.near_plane[2] = t - sv * (r0 + h)
    c.near_distance = cam.near_distance
    c.image_width, c.image_height = w, h
    return c


def timeit(scene, cam, reps=5):
    out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device=dev)
    scene.render_device(cam, 1, out.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        scene.render_device(cam, 1, out.data_ptr(), stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


res = {}
PATHS_RUN = sys.argv[1:] or ["chain", "megakernel"]
QUICK = bool(int(os.environ.get("EXP_QUICK", "0")))
for mega in PATHS_RUN:
    name = mega
    s = pkg.Scene.from_xml(xml, device=0, render_path=mega)
    cam = s.camera(0)
    res[name] = {"full": timeit(s, cam)}
    R0, C0 = (int(x) for x in os.environ.get("EXP_PIXEL", "510,1312").split(","))
    for sz in ((8,) if QUICK else (8, 16, 64, 256)):
        res[name][f"crop{sz}"] = timeit(s, crop(cam, R0 - sz // 2, C0 - sz // 2, sz, sz))
    res[name]["crop_1px"] = timeit(s, crop(cam, R0, C0, 1, 1))
    for dep in (() if QUICK else range(0, 7)):
        s.set_max_depth(dep)
        res[name][f"depth{dep}"] = timeit(s, cam)
    s.close()
print(json.dumps(res, indent=1))
