"""GPU: the bench's own timed configuration, and the workspace budget.

bench.py times C3 (horse_and_mug 1920x1080, depth 6, AA1) as one rank with 4-row
stripes, 8 hardware queues (6 workspace slots), after two 96-frame warm-up calls;
the driver runs it with --steps 20: one 20-frame rt_render_frames_device call.
Its frames go out as greedy frame batches (min(m, ceil(20 / 6)) = 4 frames
each, 4,4,4,4,4 on 5 slots) with full 32-B phase-A records (RT_COMPACT=3: a
4-frame C3 AA1 launch fits its slot's share with them; compact 16-B records
are for frame sizes that do not, such as AA2).  Every frame of that call must
be the reference's image (raytracer.cpp:505-519 renders each camera once).

RT_WS_BUDGET_MB (rt.h rt_scene_memory) bounds the scene's HBM: the uploaded scene,
its output staging and every slot's arena; a lone frame's arena follows the frame.
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


def test_bench_timed_call_equals_golden(goldens, pkg, scene_dir, torch_cuda):
    torch = torch_cuda
    g = golden_by_name(goldens, "C3_hm_1080p_d6_aa1")
    ref = torch.from_numpy(load_golden_image(g["cameras"][0]).copy()).to("cuda:0")
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        cam = s.camera(0)
        H, W = cam.image_height, cam.image_width
        bufs = torch.zeros((96, H, W, 3), dtype=torch.uint8, device="cuda:0")
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(2):                  # bench.py's warm-up calls
            s.render_frames_device([cam] * 96, 1, [b.data_ptr() for b in bufs], st, stripe_rows=4)
        torch.cuda.synchronize()
        bufs.zero_()
        before = s.counters_raw()["compact_launches"]
        s.render_frames_device([cam] * 20, 1, [bufs[i].data_ptr() for i in range(20)], st, stripe_rows=4)
        s.check()
        assert s.counters_raw()["compact_launches"] == before, "the timed call's launches must use full records"
        for i in range(20):
            assert torch.equal(bufs[i], ref), f"frame {i} of the timed call"
        # and the lone frame after it (bench's single_frame)
        s.render_device(cam, 1, bufs[0].data_ptr(), st, stripe_rows=4)
        s.check()
        assert torch.equal(bufs[0], ref)


def test_workspace_within_budget(goldens, pkg, scene_dir, torch_cuda, monkeypatch):
    """A budget-limited scene (1 GiB for C3: fewer frames per launch than the default) keeps the scene,
    its staging and every slot's arena within RT_WS_BUDGET_MB after frame batches and lone frames."""
    torch = torch_cuda
    monkeypatch.setenv("RT_WS_BUDGET_MB", "1024")
    g = golden_by_name(goldens, "C3_hm_1080p_d6_aa1")
    ref = torch.from_numpy(load_golden_image(g["cameras"][0]).copy()).to("cuda:0")
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        cam = s.camera(0)
        H, W = cam.image_height, cam.image_width
        bufs = torch.zeros((30, H, W, 3), dtype=torch.uint8, device="cuda:0")
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(2):
            s.render_frames_device([cam] * 30, 1, [b.data_ptr() for b in bufs], st, stripe_rows=H)
        s.check()
        for i in range(30):
            assert torch.equal(bufs[i], ref), f"frame {i}"
        img, _ = s.render(cam, aa=1)
        assert torch.equal(torch.from_numpy(img).to("cuda:0"), ref)
        m = s.memory()
        assert m["scene_bytes"] + m["workspace_bytes"] <= 1024 << 20, m
        # host-output staging beyond the 64 MB reserve (rt_render_cameras: 16 C3 frames, 100 MB) comes off
        # the arenas' budget too
        imgs, _ = s.render_cameras([cam] * 16, aa=1)
        for i, im in enumerate(imgs):
            assert torch.equal(torch.from_numpy(im).to("cuda:0"), ref), f"camera frame {i}"
        m = s.memory()
        assert m["scene_bytes"] + m["workspace_bytes"] <= 1024 << 20, m


def test_lone_frame_workspace(goldens, pkg, scene_dir, torch_cuda):
    """A drop-in caller (rt_render only) holds a workspace sized to its frame: <= 2 GB for C3."""
    g = golden_by_name(goldens, "C3_hm_1080p_d6_aa1")
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        for _ in range(2):
            img, _ = s.render(s.camera(0), aa=1)
        assert (img == load_golden_image(g["cameras"][0])).all()
        m = s.memory()
        assert m["workspace_bytes"] <= 2_000_000_000, m
