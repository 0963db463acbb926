"""GPU parity: the HIP path (through the C-ABI) against the reference goldens.

Bar (BASELINE.json north_star): integer RGB bit-exact after the same
clamp/quantise/SSAA; primary hit-t within 1e-4 (we also report exact-bit
agreement); work counters equal to the oracle's (same traversal order).
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import GOLDEN_DIR, config_path, golden_by_name, load_golden_image

PATHS = ["chain"]
from test_oracle import CPU_GOLDENS

pytestmark = pytest.mark.gpu

T_TOL = 1e-4   # north_star: float hit-t within 1e-4


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()
    return torch


def _counters(c):
    return (c["primary"], c["shadow"], c["reflection"], c["node_visits"], c["tri_tests"], c["sphere_tests"])


def _stats(s):
    return (s["primary_rays"], s["shadow_rays"], s["reflection_rays"], s["node_visits"], s["tri_tests"],
            s["sphere_tests"])


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("name", CPU_GOLDENS)
def test_render_bit_exact(name, path, goldens, pkg, scene_dir, torch_cuda):
    g = golden_by_name(goldens, name)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0, render_path=path) as s:
        cams = s.cameras()
        for cam in g["cameras"]:
            c, _ = cams[cam["camera"]]
            img, st = s.render(c, aa=g["aa"], stats=True)
            ref = load_golden_image(cam)
            bad = int((img != ref).any(axis=2).sum())
            assert bad == 0, f"{name}/{cam['image']}: {bad} pixels differ (max |d| " \
                             f"{int(np.abs(img.astype(int) - ref).max())})"
            assert _stats(st) == _counters(cam["counters"]), f"{name}: work counters differ from oracle"
            # the non-counting (bench) kernel variant must produce the same bytes
            img2, _ = s.render(c, aa=g["aa"], stats=False)
            assert np.array_equal(img2, ref)


@pytest.mark.parametrize("name", ["C1_simple_aa1", "C2_cornellbox_800_d0_aa1", "hm_verbatim_aa1",
                                  "C3_hm_1080p_d6_aa1"])
@pytest.mark.parametrize("walk", ["production", "reference"])
def test_primary_hit_t(name, walk, goldens, pkg, scene_dir, torch_cuda):
    """north_star's hit-t bar against the compiled reference's dump (Ray::getFirstIntersection,
    raytracer.cpp:177-225).  walk="production": the TIMED walk -- one frame through the production kernels,
    k_chain storing each sample's level-0 tSmall and material where it records its hit (k_fallback for the
    rays the timed walks defer); "reference": the side kernel's binary-tree walk, a second check."""
    g = golden_by_name(goldens, name)
    z = np.load(GOLDEN_DIR / g["primary_hits"]["file"], allow_pickle=False)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        t, m = s.primary_hits(s.camera(0), aa=g["aa"], walk=walk)
        if walk == "production":       # the dump's frame went through the production kernels' whole sequence
            s.check()
    ft, fm = t.reshape(-1), m.reshape(-1)
    assert not np.isnan(ft).any() and (fm >= 0).all(), "a sample's level-0 hit was never recorded"
    assert np.array_equal(fm[z["idx"]], z["material"])
    d = np.abs(ft[z["idx"]] - z["t"])
    assert np.max(d) <= T_TOL
    exact = float(np.mean(ft[z["idx"]].view(np.uint32) == z["t"].astype(np.float32).view(np.uint32)))
    print(f"{name} {walk}: max |dt| {float(np.max(d)):.3g}, bit-exact fraction {exact:.6f} of {len(z['idx'])}")
    # stronger than the bar: the full-frame t array is bit-identical
    assert hashlib.sha256(ft.tobytes()).hexdigest() == g["primary_hits"]["sha256_t"]
    assert hashlib.sha256(fm.tobytes()).hexdigest() == g["primary_hits"]["sha256_material"]


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("nranks,stripe,gname", [(2, 8, "C3_hm_1080p_d6_aa1"), (3, 8, "C3_hm_1080p_d6_aa1"),
                                                 (8, 8, "C3_hm_1080p_d6_aa1"), (4, 5, "C3_hm_1080p_d6_aa1"),
                                                 (3, 8, "C3_hm_1080p_d6_aa2")])
def test_stripes_unshuffle_equals_full_frame(nranks, stripe, gname, path, goldens, pkg, scene_dir, torch_cuda):
    """The multi-GPU partition rendered rank by rank on one GPU + device unshuffle."""
    torch = torch_cuda
    g = golden_by_name(goldens, gname)
    ref = load_golden_image(g["cameras"][0])
    aa = g["aa"]
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0, render_path=path) as s:
        cam = s.camera(0)
        W, H = cam.image_width, cam.image_height
        rows = pkg.slab_rows(H, stripe, nranks)
        assert rows == pkg.stripes.slab_rows(H, stripe, nranks)
        slabs = torch.zeros((nranks, rows, W, 3), dtype=torch.uint8, device="cuda:0")
        stream = torch.cuda.current_stream().cuda_stream
        for r in range(nranks):
            s.render_device(cam, aa, slabs[r].data_ptr(), stream, stripe_rows=stripe, rank=r, nranks=nranks)
        img = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
        pkg.unshuffle_stripes(slabs.data_ptr(), img.data_ptr(), W, H, stripe, nranks, stream)
        torch.cuda.synchronize()
        got = img.cpu().numpy()
        assert np.array_equal(got, ref)
        # host mirror of the mapping agrees with the device kernel
        assert np.array_equal(pkg.stripes.unshuffle(slabs.cpu().numpy(), H, stripe), ref)


@pytest.mark.parametrize("path", PATHS)
def test_device_counters_accumulate(path, goldens, pkg, scene_dir, torch_cuda):
    torch = torch_cuda
    g = golden_by_name(goldens, "C2_cornellbox_800_d0_aa1")
    cam_g = g["cameras"][0]
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0, render_path=path) as s:
        cam = s.camera(0)
        out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device="cuda:0")
        stream = torch.cuda.current_stream().cuda_stream
        s.counters_reset(stream)
        s.render_device(cam, 1, out.data_ptr(), stream, count=True)
        s.render_device(cam, 1, out.data_ptr(), stream, count=True)
        st = s.counters_read()
        assert _stats(st) == tuple(2 * v for v in _counters(cam_g["counters"]))
        assert np.array_equal(out.cpu().numpy(), load_golden_image(cam_g))


@pytest.mark.parametrize("gname", ["C3_hm_1080p_d6_aa1", "cornellbox_aa1", "C1_simple_aa1"])
def test_skipped_shadow_rays(gname, goldens, pkg, scene_dir, torch_cuda, monkeypatch):
    """Shadow rays whose light is behind the surface are not traced by the chain path
    (pathchain.hip light_needed): the image is the golden with and without the skip (RT_CULL=0), the
    counting pass still reports the reference's shadow rays, and a production counting pass
    (RT_DEBUG 0x20, which skips them) reports the same totals and the same number skipped."""
    g = golden_by_name(goldens, gname)
    cam_g = g["cameras"][0]
    ref = load_golden_image(cam_g)
    st = {}
    for cull in ("1", "0"):
        for prod in ("0", "1"):
            monkeypatch.setenv("RT_CULL", cull)
            if prod == "1":
                monkeypatch.setenv("RT_DEBUG", "0x20")      # production-fetch counting passes
            else:
                monkeypatch.delenv("RT_DEBUG", raising=False)
            with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0, render_path="chain") as s:
                c, _ = s.cameras()[cam_g["camera"]]
                img, st[cull, prod] = s.render(c, aa=g["aa"], stats=True)
                assert np.array_equal(img, ref), f"RT_CULL={cull} production counting={prod}"
                img2, _ = s.render(c, aa=g["aa"], stats=False)
                assert np.array_equal(img2, ref), f"RT_CULL={cull} (timed kernels)"
    ref_counts = _counters(cam_g["counters"])
    assert _stats(st["1", "0"]) == ref_counts
    assert _stats(st["0", "0"]) == ref_counts
    for cull in ("1", "0"):
        assert st[cull, "1"]["primary_rays"] == ref_counts[0]
        assert st[cull, "1"]["shadow_rays"] == ref_counts[1]
    assert st["0", "0"]["shadow_rays_skipped"] == 0 and st["0", "1"]["shadow_rays_skipped"] == 0
    assert st["1", "1"]["shadow_rays_skipped"] == st["1", "0"]["shadow_rays_skipped"]
    if gname.startswith("C3"):
        assert st["1", "0"]["shadow_rays_skipped"] > 0.05 * ref_counts[1]


def test_max_depth_override_matches_derived_scene(goldens, pkg, scene_dir, torch_cuda):
    """cornellbox.xml camera 2 with MaxRecursionDepth forced to 0 == the C2 golden."""
    g = golden_by_name(goldens, "C2_cornellbox_800_d0_aa1")
    with pkg.Scene.from_xml(config_path(scene_dir, "cornellbox.xml"), device=0) as s:
        s.set_max_depth(0)
        img, _ = s.render(s.camera(1), aa=1)
    assert np.array_equal(img, load_golden_image(g["cameras"][0]))


def _extra_lights(xml, n):
    """The scene with n more point lights (positions/intensities spread around the first)."""
    extra = "".join(
        f'<PointLight id="{100 + i}"><Position>{-3 + 1.5 * i} {2 + 0.5 * i} {1 - i}</Position>'
        f"<Intensity>{900 * (i + 1)} {700 * (i + 2)} {500 * (i + 3)}</Intensity></PointLight>\n"
        for i in range(n))
    return xml.replace("</Lights>", extra + "</Lights>", 1)


@pytest.mark.parametrize("path", PATHS)
def test_edge_scenes_vs_oracle(path, pkg, oracle, tmp_path, torch_cuda):
    """Empty object list (all background), negative depth (all black), odd sizes, AA 5."""
    base = pkg.scenes.scene_text("simple.xml")
    empty = base.split("<Objects>")[0] + "<Objects>\n</Objects>\n</Scene>\n"
    cases = {
        "empty": pkg.scenes.derive_xml(empty, res=(37, 23)),
        "neg_depth": pkg.scenes.derive_xml(base, depth=-1, res=(17, 9)),
        "odd_aa5": pkg.scenes.derive_xml(base, res=(33, 19)),
        "mirror_odd": pkg.scenes.derive_xml(pkg.scenes.scene_text("mirror_spheres.xml"), res=(61, 45)),
        # > 4 lights: k_finish_any (materials / lights from global memory, byte-wise occlusion)
        "six_lights": pkg.scenes.derive_xml(_extra_lights(pkg.scenes.scene_text("mirror_spheres.xml"), 5),
                                            res=(41, 37)),
    }
    for name, xml in cases.items():
        p = tmp_path / f"{name}.xml"
        p.write_text(xml.replace('<BackgroundColor>0 0 0</BackgroundColor>',
                                 '<BackgroundColor>7 200 31</BackgroundColor>'))
        aa = 5 if name == "odd_aa5" else 1
        ref, _ = oracle.OracleScene(p).render(0, aa=aa)
        with pkg.Scene.from_xml(p, device=0, render_path=path) as s:
            img, _ = s.render(s.camera(0), aa=aa)
        assert np.array_equal(img, ref), name


@pytest.mark.parametrize("name", ["C2_cornellbox_800_d0_aa1", "C3_hm_1080p_d6_aa1", "C3_hm_1080p_d6_aa2"])
def test_render_scene_from_desc(name, goldens, pkg, torch_cuda):
    """The primary constructor (rt_scene_create over borrowed host arrays in the reference's
    flattening order, raytracer.cpp:335-350) rendered on the GPU through rt_render and
    rt_render_device: bit-exact against the goldens, counters equal to the reference's."""
    torch = torch_cuda
    g = golden_by_name(goldens, name)
    arrays = pkg.scenes.scene_arrays(pkg.scenes.config_xml(g["config"]))
    with pkg.Scene.from_desc(arrays, device=0) as s:
        for cam_g in g["cameras"]:
            cam = pkg.camera_from(arrays["cameras"][cam_g["camera"]])
            ref = load_golden_image(cam_g)
            img, st = s.render(cam, aa=g["aa"], stats=True)
            assert np.array_equal(img, ref)
            assert _stats(st) == _counters(cam_g["counters"])
            img2, _ = s.render(cam, aa=g["aa"])
            assert np.array_equal(img2, ref)
            out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.uint8, device="cuda:0")
            s.render_device(cam, g["aa"], out.data_ptr(), torch.cuda.current_stream().cuda_stream)
            s.check()
            assert np.array_equal(out.cpu().numpy(), ref)


def test_bad_arguments_fail_loudly(pkg, scene_dir, torch_cuda):
    with pkg.Scene.from_xml(config_path(scene_dir, "simple.xml"), device=0) as s:
        cam = s.camera(0)
        with pytest.raises(pkg.RtError):
            s.render(cam, aa=0)
        with pytest.raises(pkg.RtError):
            s.render_device(cam, 1, 0)      # NULL output
        with pytest.raises(pkg.RtError):
            s.render_device(cam, 1, 1 << 20, stripe_rows=8, rank=3, nranks=2)


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("name", ["C5_hm_8k_d6_aa4"])
def test_full_size_c5_sha(name, path, goldens, pkg, scene_dir, torch_cuda):
    """BASELINE config 5 at full size (7680x4320, 16 spp): sha256 of the RGB bytes."""
    g = golden_by_name(goldens, name)
    cam_g = g["cameras"][0]
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0, render_path=path) as s:
        img, st = s.render(s.camera(0), aa=4, stats=True)
        # the non-counting (production) variant: closest hit on the reference-order wide tree, any
        # hit on the occlusion tree (traverse2.hpp), exact by construction -- the same bytes
        img2, _ = s.render(s.camera(0), aa=4, stats=False)
    assert hashlib.sha256(img.tobytes()).hexdigest() == cam_g["sha256_rgb"]
    assert hashlib.sha256(img2.tobytes()).hexdigest() == cam_g["sha256_rgb"]
    assert _stats(st) == _counters(cam_g["counters"])


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("name", ["cornellbox_aa1", "car_aa1", "hm_verbatim_aa2"])
def test_render_cameras_batched(name, path, goldens, pkg, scene_dir, torch_cuda):
    # (f4) multi-camera batching (raytracer.cpp:505-519): every camera of the scene in one call,
    # frames concurrent on the GPU; each image bit-identical to its golden, counters summed.
    g = golden_by_name(goldens, name)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0, render_path=path) as s:
        cams = s.cameras()
        sel = [cams[c["camera"]][0] for c in g["cameras"]]
        imgs, st = s.render_cameras(sel, aa=g["aa"], stats=True)
        for cam, img in zip(g["cameras"], imgs):
            assert np.array_equal(img, load_golden_image(cam)), f"{name}/{cam['image']}"
        tot = [sum(c["counters"][k] for c in g["cameras"]) for k in
               ("primary", "shadow", "reflection", "node_visits", "tri_tests", "sphere_tests")]
        assert list(_stats(st)) == tot
        # more frames than concurrent slots (slot reuse), order kept
        many = (sel * 4)[:9]
        imgs2, _ = s.render_cameras(many, aa=g["aa"])
        for i, img in enumerate(imgs2):
            assert np.array_equal(img, load_golden_image(g["cameras"][i % len(sel)]))


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("nranks,nframes,gname", [(1, 2, "C3_hm_1080p_d6_aa1"), (8, 8, "C3_hm_1080p_d6_aa1"),
                                                  (3, 5, "C3_hm_1080p_d6_aa1"), (8, 3, "C3_hm_1080p_d6_aa2"),
                                                  (2, 17, "C3_hm_1080p_d6_aa1")])
def test_render_frames_device_batch(nranks, nframes, gname, path, goldens, pkg, scene_dir, torch_cuda):
    """Frame batches (rt_render_frames_device, the bench's in-flight frames): every rank's stripes
    of every frame of one batched launch equal the golden, and the work counters are exactly
    nframes times the frame's (no frame's work is shared or skipped).  nframes 17 > kMaxFrames
    (two batches on two slots)."""
    torch = torch_cuda
    g = golden_by_name(goldens, gname)
    ref = load_golden_image(g["cameras"][0])
    aa, stripe = g["aa"], 8
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0, render_path=path) as s:
        cam = s.camera(0)
        W, H = cam.image_width, cam.image_height
        rows = pkg.slab_rows(H, stripe, nranks)
        slabs = torch.zeros((nframes, nranks, rows, W, 3), dtype=torch.uint8, device="cuda:0")
        stream = torch.cuda.current_stream().cuda_stream
        s.counters_reset(stream)
        for r in range(nranks):
            s.render_frames_device([cam] * nframes, aa, [slabs[f, r].data_ptr() for f in range(nframes)], stream,
                                   stripe_rows=stripe, rank=r, nranks=nranks, count=True)
        cnt = s.counters_read()
        img = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
        for f in range(nframes):
            pkg.unshuffle_stripes(slabs[f].data_ptr(), img.data_ptr(), W, H, stripe, nranks, stream)
            torch.cuda.synchronize()
            assert np.array_equal(img.cpu().numpy(), ref), f"frame {f}"
        c = g["cameras"][0]["counters"]
        assert _stats(cnt) == tuple(nframes * x for x in _counters(c))


@pytest.mark.parametrize("gname", ["C1_simple_aa1", "C1_simple_aa3", "C2_cornellbox_800_d0_aa1",
                                   "C2_cornellbox_800_d0_aa2", "hm_verbatim_aa1", "C3_hm_1080p_d6_aa1",
                                   "C3_hm_1080p_d6_aa2", "cornellbox_aa1", "simple_reflectance_aa1",
                                   "mirror_spheres_aa1", "marbles_aa1"])
def test_render_frames_device_production(gname, goldens, pkg, scene_dir, torch_cuda):
    """The bench's own call at N = 1 with the production (timed) kernels: one rank, 4-row stripes, a
    batch of 7 frames of camera 0 (frame-batch launches: compact records, A's shadow rays through
    k_occlude where phase B exists, and without it -- depth 0, C2 -- too); every frame equals the
    golden.  (test_render_frames_device_batch checks the counting kernels' batches.)"""
    torch = torch_cuda
    g = golden_by_name(goldens, gname)
    ref = torch.from_numpy(load_golden_image(g["cameras"][0]).copy()).to("cuda:0")
    aa, stripe, nframes = g["aa"], 4, 7
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        cam = s.camera(g["cameras"][0]["camera"])
        W, H = cam.image_width, cam.image_height
        slabs = torch.zeros((nframes, H, W, 3), dtype=torch.uint8, device="cuda:0")
        stream = torch.cuda.current_stream().cuda_stream
        for rep in range(2):                     # the second call sized by the first's read-backs
            slabs.zero_()
            s.render_frames_device([cam] * nframes, aa, [slabs[f].data_ptr() for f in range(nframes)], stream,
                                   stripe_rows=stripe, rank=0, nranks=1)
            torch.cuda.synchronize()
            for f in range(nframes):
                assert torch.equal(slabs[f], ref), f"{gname} call {rep} frame {f}"


@pytest.mark.parametrize("slots", ["3", "4", "6"])
def test_render_frames_device_many_batches(slots, goldens, pkg, scene_dir, torch_cuda, monkeypatch):
    """70 frames of 8-rank shards: more frames than kMaxFrames (32) per batch and more batches than
    slots, so batches reuse slot workspaces while others run; every frame equals the golden."""
    torch = torch_cuda
    monkeypatch.setenv("RT_SLOTS", slots)
    g = golden_by_name(goldens, "C3_hm_1080p_d6_aa1")
    nranks, nframes, stripe = 8, 70, 4
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        cam = s.camera(0)
        W, H = cam.image_width, cam.image_height
        rows = pkg.slab_rows(H, stripe, nranks)
        slabs = torch.zeros((nframes, nranks, rows, W, 3), dtype=torch.uint8, device="cuda:0")
        stream = torch.cuda.current_stream().cuda_stream
        for r in range(nranks):
            s.render_frames_device([cam] * nframes, 1, [slabs[f, r].data_ptr() for f in range(nframes)], stream,
                                   stripe_rows=stripe, rank=r, nranks=nranks)
        ref = torch.from_numpy(load_golden_image(g["cameras"][0]).copy()).to("cuda:0")
        img = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
        for f in range(nframes):
            pkg.unshuffle_stripes(slabs[f].data_ptr(), img.data_ptr(), W, H, stripe, nranks, stream)
            assert torch.equal(img, ref), f"frame {f}"


def test_render_frames_device_many_cameras(goldens, pkg, scene_dir, torch_cuda):
    """12 cameras, 6 distinct, in one call (batches mixing eyes): each frame equals a lone
    rt_render_device of its camera."""
    torch = torch_cuda
    g = golden_by_name(goldens, "cornellbox_aa1")
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        base = s.cameras()[1][0]
        cams = []
        for i in range(12):
            c = pkg.Camera()
            c.position, c.gaze, c.up = base.position, base.gaze, base.up
            c.near_plane, c.near_distance = base.near_plane, base.near_distance
            c.image_width, c.image_height = base.image_width, base.image_height
            c.position.x = base.position.x + 0.01 * (i % 6)      # frames i and i+6 share a camera
            cams.append(c)
        W, H = base.image_width, base.image_height
        outs = torch.zeros((len(cams), H, W, 3), dtype=torch.uint8, device="cuda:0")
        stream = torch.cuda.current_stream().cuda_stream
        s.render_frames_device(cams, 1, [o.data_ptr() for o in outs], stream, stripe_rows=H, rank=0, nranks=1)
        one = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
        for i, c in enumerate(cams):
            s.render_device(c, 1, one.data_ptr(), stream)
            torch.cuda.synchronize()
            assert torch.equal(outs[i], one), f"frame {i}"
        assert not torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("path", PATHS)
def test_render_frames_device_mixed_cameras(path, goldens, pkg, scene_dir, torch_cuda):
    """One batch holding different cameras of one size (cornellbox's two 800x800 cameras),
    split over 2 ranks: each frame uses its own eye."""
    torch = torch_cuda
    g = golden_by_name(goldens, "cornellbox_aa1")
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0, render_path=path) as s:
        order = [i for i, c in enumerate(g["cameras"]) if (c["width"], c["height"]) == (800, 800)]
        assert len(order) == 2
        order = order + order[::-1] + order
        cams = [s.cameras()[g["cameras"][i]["camera"]][0] for i in order]
        W, H = cams[0].image_width, cams[0].image_height
        assert all((c.image_width, c.image_height) == (W, H) for c in cams)
        rows = pkg.slab_rows(H, 8, 2)
        slabs = torch.zeros((len(cams), 2, rows, W, 3), dtype=torch.uint8, device="cuda:0")
        stream = torch.cuda.current_stream().cuda_stream
        for r in range(2):
            s.render_frames_device(cams, 1, [slabs[f, r].data_ptr() for f in range(len(cams))], stream,
                                   stripe_rows=8, rank=r, nranks=2)
        img = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
        for f, ci in enumerate(order):
            pkg.unshuffle_stripes(slabs[f].data_ptr(), img.data_ptr(), W, H, 8, 2, stream)
            torch.cuda.synchronize()
            assert np.array_equal(img.cpu().numpy(), load_golden_image(g["cameras"][ci])), f"frame {f}"


def test_render_cameras_device_stream(goldens, pkg, scene_dir, torch_cuda):
    torch = torch_cuda
    g = golden_by_name(goldens, "cornellbox_aa1")
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        cams = [s.cameras()[c["camera"]][0] for c in g["cameras"]]
        outs = [torch.empty((c.image_height, c.image_width, 3), dtype=torch.uint8, device="cuda") for c in cams]
        st = torch.cuda.Stream()
        s.render_cameras_device(cams, 1, [o.data_ptr() for o in outs], st.cuda_stream)
        st.synchronize()
        for cam, o in zip(g["cameras"], outs):
            assert np.array_equal(o.cpu().numpy(), load_golden_image(cam))


def test_render_device_alternating_streams(goldens, pkg, scene_dir, torch_cuda):
    """Asynchronous renders of one scene issued back to back on two different
    non-blocking streams share the scene's workspace arena: each use waits for
    the previous one (its last-use event), so every frame equals its golden."""
    torch = torch_cuda
    g = golden_by_name(goldens, "cornellbox_aa1")
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        cams = [s.cameras()[c["camera"]][0] for c in g["cameras"]]
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        order = [0, 1, 2, 1, 0, 2, 2, 0]
        outs = [torch.empty((cams[c].image_height, cams[c].image_width, 3), dtype=torch.uint8, device="cuda")
                for c in order]
        for i, c in enumerate(order):
            s.render_device(cams[c], 1, outs[i].data_ptr(), streams[i % 2].cuda_stream)
        torch.cuda.synchronize()
        s.check()
        for i, c in enumerate(order):
            assert np.array_equal(outs[i].cpu().numpy(), load_golden_image(g["cameras"][c])), f"render {i}"


def test_render_cameras_errors(pkg, scene_dir, torch_cuda):
    with pkg.Scene.from_xml(config_path(scene_dir, "simple.xml"), device=0) as s:
        with pytest.raises(pkg.RtError):
            s.render_cameras([], aa=1)
        c = s.camera(0)
        with pytest.raises(pkg.RtError):
            s.render_cameras([c], aa=0)


@pytest.mark.parametrize("name", ["cornellbox_aa1", "car_aa1"])
def test_cli_drop_in_writes_reference_ppms(name, goldens, pkg, scene_dir, tmp_path, torch_cuda):
    # the drop-in `raytracer scene.xml` (raytracer.cpp:487-525): every camera's ImageName in CWD,
    # byte-identical to the reference's write_ppm output (ppm.cpp:4-39)
    import subprocess

    g = golden_by_name(goldens, name)
    r = subprocess.run([str(pkg.CLI_PATH), str(config_path(scene_dir, g["config"])), "--aa", str(g["aa"])],
                       cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Rendered in" in r.stdout
    for cam in g["cameras"]:
        data = (tmp_path / cam["image"]).read_bytes()
        assert hashlib.sha256(data).hexdigest() == cam["sha256_ppm"], cam["image"]


@pytest.mark.parametrize("cap", [0, 5, 64])
@pytest.mark.parametrize("name", ["C3_hm_1080p_d6_aa1", "mirror_spheres_aa1"])
def test_phase_b_shadow_queue_spill(name, cap, goldens, pkg, scene_dir, torch_cuda, monkeypatch):
    # phase-B shadow tasks beyond the workgroup LDS queue spill to the global queue (k_pack_b +
    # k_occlude); tiny caps force partial reservations and SKIP slots: images and counts unchanged
    monkeypatch.setenv("RT_BQ_CAP", str(cap))
    g = golden_by_name(goldens, name)
    with pkg.Scene.from_xml(config_path(scene_dir, g["config"]), device=0) as s:
        cams = s.cameras()
        for cam in g["cameras"]:
            c, _ = cams[cam["camera"]]
            img, st = s.render(c, aa=g["aa"], stats=True)
            assert np.array_equal(img, load_golden_image(cam))
            assert _stats(st) == _counters(cam["counters"])
            img2, _ = s.render(c, aa=g["aa"], stats=False)
            assert np.array_equal(img2, load_golden_image(cam))
