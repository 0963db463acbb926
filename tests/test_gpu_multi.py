"""GPU: the C-ABI's multi-GPU device group (rt_set_devices, rt_multi.cpp) --
row stripes rendered per device, ONE (grouped) ncclGather of the uint8 slabs to
device 0, un-interleave, D2H.  On a one-GPU box:
  * the group of one device runs the whole path with RCCL (replica set-up,
    communicator, gather, unshuffle, counters);
  * RT_GROUP_VIRTUAL=1 groups of 2 and 3 ranks, all on device 0, run every part
    of the N > 1 path (replicas, per-rank streams and slabs, rank-major stripe
    mapping, frame batches, unshuffle of n slabs, summed counters) except the
    RCCL call itself, which device copies replace.
The RCCL gather at N > 1 is UNVERIFIED on hardware here (no multi-GPU box is
available to this suite).  Every image must equal the reference golden
(raytracer.cpp:487-525 renders, ppm.cpp:4-39 bytes).
"""
from __future__ import annotations

import hashlib
import subprocess

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


@pytest.fixture
def group(pkg, torch_cuda):
    """Scenes created inside the fixture form a device group over every visible GPU."""
    n = pkg.device_count()
    pkg.set_devices(n)
    yield n
    pkg.set_devices(0)


def _stats(s):
    return (s["primary_rays"], s["shadow_rays"], s["reflection_rays"], s["node_visits"], s["tri_tests"],
            s["sphere_tests"])


def _counters(c):
    return (c["primary"], c["shadow"], c["reflection"], c["node_visits"], c["tri_tests"], c["sphere_tests"])


@pytest.mark.parametrize("stripe", ["4", "8", "3"])
@pytest.mark.parametrize("name", ["C3_hm_1080p_d6_aa1", "C3_hm_1080p_d6_aa2", "cornellbox_aa1", "C1_simple_aa3"])
def test_group_render_equals_golden(name, stripe, group, goldens, pkg, scene_dir, monkeypatch):
    monkeypatch.setenv("RT_GROUP_STRIPE", stripe)
    g = golden_by_name(goldens, name)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"])) as s:
        assert s.num_devices() == group
        cams = s.cameras()
        for cam in g["cameras"]:
            c, _ = cams[cam["camera"]]
            img, st = s.render(c, aa=g["aa"], stats=True)
            assert np.array_equal(img, load_golden_image(cam)), cam["image"]
            assert _stats(st) == _counters(cam["counters"])          # summed over the devices
            img2, _ = s.render(c, aa=g["aa"])
            assert np.array_equal(img2, load_golden_image(cam))


def test_group_render_cameras_and_depth_override(group, goldens, pkg, scene_dir):
    g = golden_by_name(goldens, "cornellbox_aa1")
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"])) as s:
        cams = [c for c, _ in s.cameras()]
        imgs, st = s.render_cameras(cams, aa=1, stats=True)
        for cam in g["cameras"]:
            assert np.array_equal(imgs[cam["camera"]], load_golden_image(cam))
        assert st["primary_rays"] == sum(c["counters"]["primary"] for c in g["cameras"])
    # MaxRecursionDepth override reaches every replica: C3 scene at depth 2 on the group = the same
    # scene at depth 2 on one device without a group
    with pkg.Scene.from_xml(config_path(scene_dir, "C3_hm_1080p_d6")) as s:
        s.set_max_depth(2)
        a, _ = s.render(s.camera(0), aa=1)
    pkg.set_devices(0)
    with pkg.Scene.from_xml(config_path(scene_dir, "C3_hm_1080p_d6"), device=0, render_path="chain") as one:
        assert one.num_devices() == 1
        one.set_max_depth(2)
        b, _ = one.render(one.camera(0), aa=1)
    assert np.array_equal(a, b)


@pytest.fixture(params=[2, 3])
def virtual_group(request, pkg, torch_cuda, monkeypatch):
    """A rehearsal group of 2 or 3 ranks on device 0 (RT_GROUP_VIRTUAL: copies instead of RCCL)."""
    monkeypatch.setenv("RT_GROUP_VIRTUAL", "1")
    pkg.set_devices(request.param)
    yield request.param
    pkg.set_devices(0)


@pytest.mark.parametrize("stripe,batch", [("4", None), ("8", None), ("5", None), ("4", "1")])
def test_virtual_group_frames_equal_golden(virtual_group, stripe, batch, goldens, pkg, scene_dir, monkeypatch):
    """N > 1 group path on one GPU: single frames (rt_render) and frame batches (rt_render_cameras:
    every rank renders its stripes of a run of same-size cameras in flight together, one grouped
    gather, per-frame unshuffle) equal the goldens; counters are summed over the ranks.
    RT_GROUP_BATCH=1: the escape hatch, one frame (one gather) per call."""
    monkeypatch.setenv("RT_GROUP_STRIPE", stripe)
    if batch:
        monkeypatch.setenv("RT_GROUP_BATCH", batch)
    g = golden_by_name(goldens, "C3_hm_1080p_d6_aa1")
    cam_g = g["cameras"][0]
    ref = load_golden_image(cam_g)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"])) as s:
        assert s.num_devices() == virtual_group
        img, st = s.render(s.camera(0), aa=1, stats=True)
        assert np.array_equal(img, ref)
        assert _stats(st) == _counters(cam_g["counters"])
        imgs, st = s.render_cameras([s.camera(0)] * 3, aa=1, stats=True)
        for im in imgs:
            assert np.array_equal(im, ref)
        assert _stats(st) == tuple(3 * v for v in _counters(cam_g["counters"]))
    g = golden_by_name(goldens, "cornellbox_aa1")
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"])) as s:
        cams = [c for c, _ in s.cameras()]
        order = [1, 2, 0, 2, 1]             # mixed sizes (480^2, 800^2): runs of same-size frames
        imgs, _ = s.render_cameras([cams[i] for i in order], aa=1)
        for i, im in zip(order, imgs):
            cam = next(c for c in g["cameras"] if c["camera"] == i)
            assert np.array_equal(im, load_golden_image(cam))


@pytest.mark.parametrize("name", ["cornellbox_aa1", "car_aa1"])
def test_cli_gpus_writes_reference_ppms(name, goldens, pkg, scene_dir, tmp_path, torch_cuda):
    """The drop-in CLI with --gpus (rt_set_devices before the scene load)."""
    g = golden_by_name(goldens, name)
    n = pkg.device_count()
    r = subprocess.run([str(pkg.CLI_PATH), str(config_path(scene_dir, g["config"])), "--aa", str(g["aa"]),
                        "--gpus", str(n)], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert f"on {n} GPU(s)" in r.stdout
    for cam in g["cameras"]:
        data = (tmp_path / cam["image"]).read_bytes()
        assert hashlib.sha256(data).hexdigest() == cam["sha256_ppm"], cam["image"]


def test_set_devices_errors(pkg, torch_cuda):
    with pytest.raises(pkg.RtError):
        pkg.set_devices(-1)
    with pytest.raises(pkg.RtError):
        pkg.set_devices(pkg.device_count() + 1)
    pkg.set_devices(0)
