"""Wave-step statistics of the walk loops (diagnostics build, RT_STEP_STATS=1):
   make BUILD=build_stats LIB=librt_stats.so EXTRA=-DRT_STEP_STATS=1 librt_stats.so
   RT_LIB=raytracer-ceng477-graphics-hw-1_amd/librt_stats.so python tools/step_stats.py [config] [frames]
Prints, per role, wave iterations, average walking lanes per iteration, lanes at interior nodes /
leaf records, the fraction of iterations that issue both step kinds, and refills."""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "raytracer-ceng477-graphics-hw-1_amd"))
import __graft_entry__ as g  # noqa: E402
import scenes  # noqa: E402

pkg = g.import_pkg()
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3_hm_1080p_d6"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 1
L = pkg.lib()
fn = L.rt_debug_step_stats
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 32)()
path = scenes.write_config(cfg, "/tmp/step_stats")
with pkg.Scene.from_xml(path, device=0) as s:
    cam = s.camera(0)
    outs = [torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device="cuda") for _ in range(frames)]
    st = torch.cuda.current_stream().cuda_stream
    for rep in range(2):            # warm, then measured
        assert fn(buf, 1) == 1, "not an RT_STEP_STATS build"
        if frames == 1:
            s.render_device(cam, 1, outs[0].data_ptr(), st)
        else:
            s.render_frames_device([cam] * frames, 1, [o.data_ptr() for o in outs], st)
        torch.cuda.synchronize()
    fn(buf, 0)
v = np.array(list(buf), dtype=np.float64).reshape(4, 8)
for role, name in enumerate(["phase-A chains", "phase-B chains", "shadow (k_mix/k_occlude)", "shadow (phase-B queue)"]):
    it, walk, inner, leaf, leaf_it, ref, reflanes, inner_it = v[role] / frames
    if it == 0:
        continue
    print(f"{name:26s} iter {it / 1e6:6.3f}M walking {walk / it:4.1f}/64 | interior: {inner_it / it:4.2f} of iter, "
          f"{inner / max(inner_it, 1):4.1f} lanes | leaf: {leaf_it / it:4.2f} of iter, {leaf / max(leaf_it, 1):4.1f} lanes"
          f" | refills {ref / 1e3:6.1f}K x {reflanes / max(ref, 1):4.1f} lanes")
