"""GPU: a lone frame's phase-A units dealt by the previous frame's costs (pathchain.hip rank_units: seven
cost classes, heaviest first).  Only where work runs changes: every repeated frame must equal the
reference's image -- ranked or not, with the mixed deal of the heaviest units (PcParams::ugrp), with the
phase-B record space cut, with the LDS shadow queue off and with every shadow ray deferred to k_fallback.
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
    {"RT_HOT_UNITS": "1"},
    {"RT_HOT_UNITS": "0"},
    {"RT_HOT_UNITS": "1", "RT_CONT_CB": "2000"},             # most continuations beyond the record space
    {"RT_HOT_UNITS": "1", "RT_BQ_CAP": "0"},
    {"RT_HOT_UNITS": "1", "RT_FORCE_FALLBACK": "2"},
    {"RT_HOT_UNITS": "1", "RT_MIX": "0"},                    # heaviest first, no mixed deal
    {"RT_HOT_UNITS": "1", "RT_MIX": "5"},                    # mixed deal, G from the hot-unit count and the grid
    {"RT_HOT_UNITS": "1", "RT_MIX": str(6 | 1 << 8)},        # every marked class, G = 2
    {"RT_HOT_UNITS": "1", "RT_MIX": str(1 | 3 << 8), "RT_CONT_CB": "2000"},   # G = 8, record space cut
]


@pytest.mark.parametrize("env", ENVS, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
@pytest.mark.parametrize("name", ["C3_hm_1080p_d6_aa1", "mirror_spheres_aa1", "marbles_aa1", "C1_simple_aa2",
                                  "hm_verbatim_aa2", "cornellbox_aa1"])
def test_hot_units_bit_exact(name, env, goldens, pkg, scene_dir, torch_cuda, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = golden_by_name(goldens, name)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        cams = s.cameras()
        for rep in range(3):                     # frame 2 on: dealt by the previous frame's costs
            for cam in g["cameras"]:
                c, _ = cams[cam["camera"]]
                img, _ = s.render(c, aa=g["aa"])
                bad = int((img != load_golden_image(cam)).any(axis=2).sum())
                assert bad == 0, f"{name}/{cam['image']} {env} frame {rep}: {bad} pixels differ"
