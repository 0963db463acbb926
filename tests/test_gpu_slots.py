"""GPU: the workspace slots and arenas at HIP's DEFAULT queue count.

The suite (conftest.py), bench.py and the CLI run with 8 hardware queues, so the
library runs 6 workspace slots.  An ordinary C-ABI or Python caller gets HIP's
default of 4 queues and therefore 3 slots (rt_api.cpp tune_slots).  This runs the
slot/arena paths in a child process started with GPU_MAX_HW_QUEUES=4 (the
variable is read when HIP starts): frame batches on several slots, slot reuse,
multi-camera batches and frame chunks on slot streams, each image against its
golden (raytracer.cpp:505-519 renders one camera after another).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
import numpy as np, torch
import __graft_entry__ as graft
from conftest import golden_by_name, load_golden_image, GOLDEN_DIR
pkg = graft.import_pkg()
goldens = json.loads((GOLDEN_DIR / "goldens.json").read_text())["goldens"]
import tempfile
d = tempfile.mkdtemp()
out = {}
g = golden_by_name(goldens, "C3_hm_1080p_d6_aa1")
ref = load_golden_image(g["cameras"][0])
with pkg.Scene.from_xml(pkg.scenes.write_config("C3_hm_1080p_d6", d), device=0) as s:
    cam = s.camera(0)
    H, W = cam.image_height, cam.image_width
    bufs = torch.empty((14, H, W, 3), dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    s.render_frames_device([cam] * 14, 1, [bufs[i].data_ptr() for i in range(14)], st, stripe_rows=H)
    s.check()
    out["frames_ok"] = all(np.array_equal(bufs[i].cpu().numpy(), ref) for i in range(14))
    imgs, _ = s.render_cameras([cam] * 5, aa=1)
    out["cameras_ok"] = all(np.array_equal(im, ref) for im in imgs)
    one, _ = s.render(cam, aa=1)
    out["single_ok"] = np.array_equal(one, ref)
g = golden_by_name(goldens, "cornellbox_aa1")
with pkg.Scene.from_xml(pkg.scenes.write_config("cornellbox.xml", d), device=0) as s:
    cams = s.cameras()
    sel = [cams[c["camera"]][0] for c in g["cameras"]] * 3
    imgs, _ = s.render_cameras(sel, aa=1)
    out["cornell_ok"] = all(np.array_equal(im, load_golden_image(g["cameras"][i % len(g["cameras"])]))
                            for i, im in enumerate(imgs))
print(json.dumps(out))
"""


def test_slots_at_default_queue_count():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, GPU_MAX_HW_QUEUES="4")
    env.pop("RT_HW_QUEUES", None)
    env.pop("RT_SLOTS", None)
    r = subprocess.run([sys.executable, "-c", CHILD, str(ROOT)], env=env, capture_output=True, text=True,
                       timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res == {"frames_ok": True, "cameras_ok": True, "single_ok": True, "cornell_ok": True}, res
