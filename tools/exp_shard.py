#!/usr/bin/env python3
"""Experiment: per-rank render time of the C3 frame's row-stripe shards, on ONE GPU.

For world sizes N and stripe heights S, renders rank r's stripes (r = 0..N-1,
one after another on the same GPU) and reports the median kernel time of each
rank and the max over ranks.  The max is what a real N-GPU run waits for
before its gather, so this predicts strong-scaling efficiency without an
N-GPU node (the gather itself is not included).

  python tools/exp_shard.py [N ...]      (default 1 2 4 8; env EXP_S="1 2 4 8 16")
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
sp = stream.cuda_stream
scene = pkg.Scene.from_xml(xml, device=0)
cam = scene.camera(0)
W, H = cam.image_width, cam.image_height
worlds = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]
stripes = [int(x) for x in os.environ.get("EXP_S", "8").split()]
reps = int(os.environ.get("EXP_REPS", "7"))


F = int(os.environ.get("EXP_F", "1"))     # frames in flight (rt_render_frames_device); time per frame


def time_rank(S, r, N):
    rows = pkg.slab_rows(H, S, N)
    outs = [torch.empty((rows, W, 3), dtype=torch.uint8, device=dev) for _ in range(F)]

    def go():
        if F == 1:
            scene.render_device(cam, 1, outs[0].data_ptr(), sp, S, r, N)
        else:
            scene.render_frames_device([cam] * F, 1, [o.data_ptr() for o in outs], sp, S, r, N)
    for _ in range(2):
        go()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        go()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / F)
    return sorted(ts)[len(ts) // 2]


res = []
for S in stripes:
    for N in worlds:
        per = [time_rank(S, r, N) for r in range(N)]
        t1 = res[0]["max_ms"] if res and res[0]["S"] == S and res[0]["N"] == 1 else None
        row = {"S": S, "N": N, "max_ms": round(max(per), 4), "min_ms": round(min(per), 4),
               "per_rank_ms": [round(x, 4) for x in per]}
        res.append(row)
        print(json.dumps(row), flush=True)
scene.close()
