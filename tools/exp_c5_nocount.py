#!/usr/bin/env python3
"""One non-counting C5 frame (7680x4320, 16 spp) through rt_render_device; prints its time."""
import sys, tempfile, time
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as graft  # noqa: E402
pkg = graft.import_pkg()
cfg = sys.argv[1] if len(sys.argv) > 1 else "C5_hm_8k_d6"
aa = int(sys.argv[2]) if len(sys.argv) > 2 else 4
xml = pkg.scenes.write_config(cfg, tempfile.mkdtemp())
s = pkg.Scene.from_xml(xml, device=0)
cam = s.camera(0)
out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
for i in range(2):
    t0 = time.perf_counter()
    s.render_device(cam, aa, out.data_ptr(), st.cuda_stream, cam.image_height, 0, 1)
    torch.cuda.synchronize()
    print(f"{cfg} aa{aa} frame {i}: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
