#!/usr/bin/env python3
"""Scene creation time on the GPU box (the drop-in CLI's "Planted trees"): XML load + host build +
upload, per call in one process (the first call also initialises HIP), beside the host-only path.

  python tools/exp_scene_load.py [config]
"""
import json
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as graft  # noqa: E402

pkg = graft.import_pkg()
xml = pkg.scenes.write_config(sys.argv[1] if len(sys.argv) > 1 else "C3_hm_1080p_d6", tempfile.mkdtemp())
res = {"device": [], "host_only": []}
for kind in ("device", "host_only", "device"):
    for _ in range(3):
        t0 = time.perf_counter()
        s = pkg.Scene.from_xml(xml, device=0) if kind == "device" else pkg.Scene.from_xml(xml, host_only=True)
        ms = (time.perf_counter() - t0) * 1e3
        b = s.bvh_info()
        s.close()
        res[kind].append({"ms": round(ms, 2), "build_ms": round(b["build_ms"], 2), "ref_ms": round(b["ref_ms"], 2),
                          "wide_ms": round(b["wide_ms"], 2), "threads": b["build_threads"]})
print(json.dumps(res))
