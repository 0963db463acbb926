#!/usr/bin/env python3
"""Multi-camera batching (rt_render_cameras_device) against one camera after
another on one stream (raytracer.cpp:505-519), device time per batch.
  python tools/exp_batch.py [scene.xml|config] [aa] [repeat-cameras]
"""
import json
import sys
import tempfile
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as graft  # noqa: E402

pkg = graft.import_pkg()
name = sys.argv[1] if len(sys.argv) > 1 else "cornellbox.xml"
aa = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rep = int(sys.argv[3]) if len(sys.argv) > 3 else 1
d = tempfile.mkdtemp()
xml = pkg.scenes.write_config(name, d)
s = pkg.Scene.from_xml(xml, device=0)
cams = [c for c, _ in s.cameras()] * rep
outs = [torch.empty((c.image_height, c.image_width, 3), dtype=torch.uint8, device="cuda") for c in cams]
st = torch.cuda.current_stream()


def seq():
    for c, o in zip(cams, outs):
        s.render_device(c, aa, o.data_ptr(), st.cuda_stream)


def bat():
    s.render_cameras_device(cams, aa, [o.data_ptr() for o in outs], st.cuda_stream)


def timeit(f, n=10):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        f()
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[n // 2]


print(json.dumps({"scene": name, "cameras": len(cams), "aa": aa, "sequential_ms": round(timeit(seq), 4),
                  "batched_ms": round(timeit(bat), 4)}))
