#!/usr/bin/env python3
"""Scene creation time on the GPU box (the drop-in CLI's "Planted trees"): XML load + host build +
upload, per call in one process (the first call also initialises HIP), with its phases
(rt_bvh_info: xml, triangle prep, reference tree, flatten, reference-order wide tree, occlusion tree,
upload), at several build thread counts, beside the host-only path.

  python tools/exp_scene_load.py [config] [threads,...]
"""
import json
import os
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as graft  # noqa: E402

pkg = graft.import_pkg()
xml = pkg.scenes.write_config(sys.argv[1] if len(sys.argv) > 1 else "C3_hm_1080p_d6", tempfile.mkdtemp())
threads = [int(t) for t in (sys.argv[2] if len(sys.argv) > 2 else "16,8,4,1").split(",")]
PH = ("build_ms", "xml_ms", "prep_ms", "ref_ms", "flat_ms", "refwide_ms", "stree_ms", "upload_ms")
res = {}
first = True
for th in threads:
    os.environ["RT_BUILD_THREADS"] = str(th)
    for kind in ("device", "host_only"):
        rows = []
        for rep in range(6):
            t0 = time.perf_counter()
            s = pkg.Scene.from_xml(xml, device=0) if kind == "device" else pkg.Scene.from_xml(xml, host_only=True)
            ms = (time.perf_counter() - t0) * 1e3
            b = s.bvh_info()
            s.close()
            if first:          # the process's first scene also initialises HIP
                first = False
                res["first_call_ms"] = round(ms, 2)
                continue
            rows.append({"ms": round(ms, 2), **{k: round(b[k], 2) for k in PH}, "threads": b["build_threads"]})
        med = sorted(r["ms"] for r in rows)[len(rows) // 2]
        res[f"{kind}_t{th}"] = {"median_ms": med, "runs": rows}
        print(f"{kind} threads={th}: median {med} ms; last {rows[-1]}", file=sys.stderr, flush=True)
print(json.dumps(res))
