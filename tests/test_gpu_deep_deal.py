"""GPU: frame batches' deep-first deal (pathchain.hip k_chain / k_pack_a, PcParams::pdepth).  A continuation
whose frame slot went at least RT_DEEP levels deep in the previous launch of the same frame geometry is queued
at its region's end and packed first, so phase B starts the long chains first.  Only the order of phase B's
work changes: every frame of every batch must still be the reference's image -- deal off, every continuation
deep (1), the default (5), none (255), with the record space cut (the rest through k_fallback), across scenes
whose frame geometry changes between calls (the depth table is cleared) and with a lone frame in between
(a whole lone frame reads its lists in place and takes no part in the deal).
"""
from __future__ import annotations

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
    {"RT_DEEP": "0"},
    {"RT_DEEP": "1"},
    {"RT_DEEP": "5"},
    {"RT_DEEP": "255"},
    {"RT_DEEP": "2", "RT_CONT_CB": "2000"},      # most continuations beyond the record space
]


@pytest.mark.parametrize("env", ENVS, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
@pytest.mark.parametrize("name", ["C3_hm_1080p_d6_aa1", "mirror_spheres_aa1", "marbles_aa1", "C1_simple_aa2",
                                  "cornellbox_aa1"])
def test_deep_deal_bit_exact(name, env, goldens, pkg, scene_dir, torch_cuda, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = golden_by_name(goldens, name)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        cams = s.cameras()
        refs = [load_golden_image(cam) for cam in g["cameras"]]
        sel = [cam for cam in g["cameras"] for _ in range(3)]
        for call in range(3):                    # call 1 on: dealt by the previous call's depths
            imgs, _ = s.render_cameras([cams[cam["camera"]][0] for cam in sel], aa=g["aa"])
            for i, (cam, img) in enumerate(zip(sel, imgs)):
                bad = int((img != refs[g["cameras"].index(cam)]).any(axis=2).sum())
                assert bad == 0, f"{name}/{cam['image']} {env} call {call} frame {i}: {bad} pixels differ"
            if call == 1:                        # a lone frame between batches
                c, _ = cams[g["cameras"][0]["camera"]]
                img, _ = s.render(c, aa=g["aa"])
                assert int((img != refs[0]).any(axis=2).sum()) == 0, f"{name} {env}: lone frame"
