#!/usr/bin/env python3
"""Diagnostics (a library built with RT_TRACE_BUILD=1, named by RT_LIB): one lone C3 frame's timeline --
phase A's samples, phase B's continuations, and every k_mix workgroup's start / chain-role end / end by role
(chain or shadow).  Times in us from the first record of each kernel (100 MHz wall clock).

  RT_LIB=.../librt_trace.so python tools/trace_mix.py [ENV=V ...]
"""
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

for kv in sys.argv[1:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
tf = os.path.join(tempfile.mkdtemp(), "trace.bin")
os.environ["RT_TRACE"] = tf
import torch  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as graft  # noqa: E402

pkg = graft.import_pkg()
xml = pkg.scenes.write_config(os.environ.get("EXP_SCENE", "C3_hm_1080p_d6"), tempfile.mkdtemp())
with pkg.Scene.from_xml(xml, device=0) as s:
    cam = s.camera(0)
    out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device="cuda:0")
    for _ in range(3):
        s.render_device(cam, 1, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
raw = np.fromfile(tf, dtype=np.uint32)
assert raw[0] == 0x52545452
_, cap, tb, n = (int(x) for x in raw[1:5])
d = raw[5:5 + n].astype(np.int64)
samp = d[:2 * cap].reshape(cap, 2)
cont = d[2 * (cap + tb):2 * (cap + tb) + 4 * cap].reshape(cap, 4)
mix = d[2 * (cap + tb) + 4 * cap:2 * (cap + tb) + 4 * cap + 4 * tb].reshape(tb, 4)


def rel(x, t0):
    return ((x - t0) & 0xffffffff) * 0.01


def pct(x):
    return {p: round(float(np.percentile(x, p)), 1) for p in (50, 90, 99, 100)} if len(x) else None


ok = samp[:, 1] != 0
tA = samp[ok, 0].min()
res = {"phaseA_end_us": pct(rel(samp[ok, 1], tA))}
m = mix[mix[:, 3] != 0]
t0 = m[:, 0].min()
res["mix_start_after_A_start_us"] = round(float(rel(np.array([t0]), tA)[0]), 1)
ch, sh = m[m[:, 3] == 1], m[m[:, 3] == 2]
res["mix_chain_wgs"] = len(ch)
res["mix_chain_role_end_us"] = pct(rel(ch[:, 1], t0))
res["mix_chain_wg_end_us"] = pct(rel(ch[:, 2], t0))
res["mix_shadow_wgs"] = len(sh)
res["mix_shadow_start_us"] = pct(rel(sh[:, 0], t0))
res["mix_shadow_end_us"] = pct(rel(sh[:, 2], t0))
c = cont[cont[:, 1] != 0]
if len(c):
    res["phaseB_cont"] = len(c)
    res["phaseB_grab_us"] = pct(rel(c[:, 0], t0))
    res["phaseB_end_us"] = pct(rel(c[:, 1], t0))
print(json.dumps(res, indent=1))
