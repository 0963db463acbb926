"""GPU: the shadow walks' wave leaf queue (pathchain.hip occlude_queue_body).

A's shadow rays (k_occlude in frame batches, k_mix's shadow role for one frame) and phase B's
overflow queue their leaf records per wave and test them 64 at a time against the owner lanes'
rays (any hit is order-free, raytracer.cpp:227-280).  These tests drive its scheduling edges and
compare with the reference goldens (raytracer.cpp:385-452):
  * RT_LQ_WAIT=1: records tested as soon as one lane waits on them (many small flushes);
  * RT_LQ_WAIT=64: only when 64 records are queued or no lane walks (the queue fills to its
    128-entry capacity and the drain stops at it);
  * RT_OREFILL=4 / 60: tasks refilled when almost none / almost all lanes hold one;
  * RT_BQ_CAP=0: every phase-B shadow ray goes through k_occlude's overflow role too.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import config_path, golden_by_name, load_golden_image

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()
    return torch


ENVS = [
    {"RT_LQ_WAIT": "1"},
    {"RT_LQ_WAIT": "64"},
    {"RT_OREFILL": "4"},
    {"RT_OREFILL": "60", "RT_LQ_WAIT": "8"},
    {"RT_BQ_CAP": "0"},
]


@pytest.mark.parametrize("env", ENVS, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
@pytest.mark.parametrize("name", ["C3_hm_1080p_d6_aa1", "cornellbox_aa1", "mirror_spheres_aa1", "C1_simple_aa2"])
def test_leaf_queue_bit_exact(name, env, goldens, pkg, scene_dir, torch_cuda, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = golden_by_name(goldens, name)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0, render_path="chain") as s:
        cams = s.cameras()
        for cam in g["cameras"]:
            c, _ = cams[cam["camera"]]
            img, _ = s.render(c, aa=g["aa"])
            bad = int((img != load_golden_image(cam)).any(axis=2).sum())
            assert bad == 0, f"{name}/{cam['image']} {env}: {bad} pixels differ"
        sel = [cams[c["camera"]][0] for c in g["cameras"]] * 2
        imgs, _ = s.render_cameras(sel, aa=g["aa"])
        for i, img in enumerate(imgs):
            assert np.array_equal(img, load_golden_image(g["cameras"][i % len(g["cameras"])])), f"batch {i} {env}"
