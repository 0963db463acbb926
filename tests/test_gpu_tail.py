"""GPU: k_tail, phase B's last chains walked one wave per chain (pathchain.hip).

Once at most RT_TAIL (lone frames) / RT_TAIL_B (frame batches) phase-B chains of
the launch are left, a k_mix chain wave with no continuation left hands its chains
on at a level boundary
(the walk it is on restarts in k_tail from its ray, the reflection of the previous
level's record).  k_tail walks the reference's ordered closest hit with the whole
wave (a lane per wide-node slot, a lane per leaf primitive, a lane per stack
entry) and runs chain_body's epilogue (raytracer.cpp:385-452): the images must be
the reference's whatever the threshold (the live chains left when the hand-off
starts) -- 0 (off), 1, 500, 2000, every chain once the continuations run out, and
RT_TAIL_ALL (every continuation handed on at its first phase-B walk: all of phase
B in k_tail), and phase A's stragglers likewise to k_tail_a (RT_TAIL_A /
RT_TAIL_A_B, the samples left once every unit is taken) --
with the phase-B record space cut (RT_CONT_CB: the rest in k_fallback), with
every shadow task of phase B through k_occlude (RT_BQ_CAP=0), and with k_mix's
A shadow tasks dealt statically or dynamically in chunks (RT_DCHUNK).
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
    {"RT_TAIL": "0", "RT_TAIL_B": "0", "RT_DCHUNK": "0"},
    {"RT_TAIL": "0", "RT_DCHUNK": "7"},                      # (raised to the smallest chunk that reaches every task)
    {"RT_TAIL": "1", "RT_TAIL_B": "1"},
    {"RT_TAIL": "2000", "RT_TAIL_B": "2000", "RT_DCHUNK": "1024"},
    {"RT_TAIL": "1000000", "RT_TAIL_B": "1000000"},          # every chain left once the waves run out of continuations
    {"RT_TAIL": "1", "RT_TAIL_B": "1", "RT_TAIL_ALL": "1"},  # every chain from its first phase-B walk
    {"RT_TAIL": "1", "RT_TAIL_B": "1", "RT_TAIL_ALL": "1", "RT_CONT_CB": "1000"},
    {"RT_TAIL": "500", "RT_BQ_CAP": "0", "RT_TAIL_GRID": "7"},
    {"RT_TAIL": "1", "RT_TAIL_ALL": "1", "RT_COMPACT": "2", "RT_TAIL_B": "1"},
    {"RT_TAIL": "1000000", "RT_OCC_INPLACE": "0"},
    # k_finish split (on with any phase-B tail in a lone frame): off; with every ray deferred to k_fallback
    # (kPathFb pixels in part 2); with the fallback shadow queue overflowing (part 2 takes every pixel)
    {"RT_TAIL": "2000", "RT_FIN_SPLIT": "0"},
    {"RT_TAIL": "2000", "RT_FORCE_FALLBACK": "2"},
    {"RT_TAIL": "2000", "RT_FORCE_FALLBACK": "3", "RT_FBS_CAP": "64"},
    {"RT_TAIL": "1", "RT_TAIL_ALL": "1", "RT_FBS_CAP": "64", "RT_FORCE_FALLBACK": "2"},
    # phase A's stragglers to k_tail_a (levels 0..1, then phase B as usual)
    {"RT_TAIL_A": "1", "RT_TAIL_A_B": "1"},
    {"RT_TAIL_A": "5000", "RT_TAIL_A_B": "5000", "RT_TAIL": "2000", "RT_TAIL_B": "2000"},
    {"RT_TAIL_A": "100000000", "RT_TAIL_A_B": "100000000"},   # every sample left once the units run out
    {"RT_TAIL_A": "1", "RT_TAIL_ALL": "1", "RT_TAIL": "1"},    # every sample from its first walk, A and B
    {"RT_TAIL_A_B": "1", "RT_TAIL_ALL": "1", "RT_COMPACT": "2", "RT_CONT_CB": "1000"},
]


@pytest.mark.parametrize("env", ENVS, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
@pytest.mark.parametrize("name", ["C3_hm_1080p_d6_aa1", "mirror_spheres_aa1", "marbles_aa1", "C1_simple_aa2"])
def test_tail_bit_exact(name, env, goldens, pkg, scene_dir, torch_cuda, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = golden_by_name(goldens, name)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        cams = s.cameras()
        for cam in g["cameras"]:
            c, _ = cams[cam["camera"]]
            ref = load_golden_image(cam)
            for rep in range(2):                  # the second frame deals phase A by the first's costs
                img, _ = s.render(c, aa=g["aa"])
                bad = int((img != ref).any(axis=2).sum())
                assert bad == 0, f"{name}/{cam['image']} {env} frame {rep}: {bad} pixels differ"
        # frame batches (RT_TAIL_B)
        sel = [cams[c["camera"]][0] for c in g["cameras"]] * 3
        imgs, _ = s.render_cameras(sel, aa=g["aa"])
        for i, img in enumerate(imgs):
            assert np.array_equal(img, load_golden_image(g["cameras"][i % len(g["cameras"])])), f"batch {i} {env}"
