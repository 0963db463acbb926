"""GPU: k_fallback, the general walker behind the timed chain kernels.

The timed kernels (k_chain, k_mix, k_occlude) walk only the wide trees; a ray
the wide trees' fused slab test does not take (NaN, or a direction component
of exactly 0) is deferred to k_fallback, which also finishes the continuations
beyond the phase-B record capacity (pathchain.hip).  These tests force every
branch of it and compare with the reference goldens (raytracer.cpp:385-452):
  * RT_FORCE_FALLBACK=1: every closest-hit ray deferred (whole paths walked,
    shaded and folded in k_fallback: tail colours, kEndTail);
  * =2: every shadow ray deferred (the fallback shadow queue);
  * =3: both;
  * =4: every reflected ray deferred (phase A records level 0, k_fallback
    walks the rest of each mirror path from level 1; its pinfo write clears
    the kPathCont bit k_chain set, so k_finish's second loop finishes the
    pixel -- ADVICE r5);
  * RT_CONT_CB=1000: continuations beyond 1,000 finish in k_fallback;
  * RT_FBS_CAP=64 with =2: the shadow queue overflows (marked occlusion bytes
    scanned by k_fallback);
  * RT_COMPACT=0 with RT_CONT_CB=1000: full 32-B phase-A records (the compact
    16-B records leave the directions of continued paths in tail[]);
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
    {"RT_FORCE_FALLBACK": "1"},
    {"RT_FORCE_FALLBACK": "2"},
    {"RT_FORCE_FALLBACK": "3"},
    {"RT_FORCE_FALLBACK": "4"},
    {"RT_CONT_CB": "1000"},
    # phase-A records with their directions (RT_COMPACT=0, pathchain.hpp dbase = 0): the continuations
    # and k_fallback read the stored direction words instead of the chain's tail copies
    {"RT_COMPACT": "0", "RT_CONT_CB": "1000"},
    {"RT_FORCE_FALLBACK": "2", "RT_FBS_CAP": "64"},
]


@pytest.mark.parametrize("env", ENVS, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
@pytest.mark.parametrize("name", ["C3_hm_1080p_d6_aa1", "cornellbox_aa1", "mirror_spheres_aa1", "C1_simple_aa2"])
def test_fallback_paths_bit_exact(name, env, goldens, pkg, scene_dir, torch_cuda, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = golden_by_name(goldens, name)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0, render_path="chain") as s:
        cams = s.cameras()
        for cam in g["cameras"]:
            c, _ = cams[cam["camera"]]
            img, _ = s.render(c, aa=g["aa"])
            ref = load_golden_image(cam)
            bad = int((img != ref).any(axis=2).sum())
            assert bad == 0, f"{name}/{cam['image']} {env}: {bad} pixels differ"
        # frame batches (several frames per launch, phase-B records by continuation index)
        sel = [cams[c["camera"]][0] for c in g["cameras"]] * 2
        imgs, _ = s.render_cameras(sel, aa=g["aa"])
        for i, img in enumerate(imgs):
            assert np.array_equal(img, load_golden_image(g["cameras"][i % len(g["cameras"])])), f"batch {i} {env}"
