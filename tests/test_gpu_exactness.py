"""GPU: the closest-hit walk over the reference-order 4-wide tree
(traverse2.hpp wide_closest_step) against the reference walk, on the rays
where a tolerance-based walk would be most fragile: grazing rays over large
flat axis-aligned patches (Cramer's t and the slab t of a zero-thickness leaf
box round differently), rays starting on the floor plane, and mirror chains
between near-parallel mirrors.  Also the always-on walk step bound.

The reference here is (a) the C oracle (rt_oracle.c, a restatement of
raytracer.cpp:177-280 pinned to the compiled reference by the goldens) for
whole images and work counters, and (b) the device's own binary reference-tree
walk (rt_walk_timing mode 1, the reference's ordered DFS over its own nodes)
for millions of single rays.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()
    return torch


def _fmt(v: float) -> str:
    return repr(float(np.float32(v)))


def grazing_scene(nx: int = 48, nz: int = 48, res=(160, 90), depth: int = 4, cam_h: float = 0.02) -> str:
    """A mirror floor of nx*nz axis-aligned quads (y = 0, two triangles each, so its BVH leaves are flat
    boxes), two facing near-parallel mirror walls, a few tilted tiles and a sphere resting on the floor;
    the camera sits cam_h above the floor looking almost along it."""
    rng = np.random.default_rng(7)
    verts, faces_floor, faces_wall, faces_tilt = [], [], [], []

    def v(x, y, z):
        verts.append((x, y, z))
        return len(verts)

    size = 8.0
    xs = np.linspace(-size, size, nx + 1)
    zs = np.linspace(-2 * size, 0.5, nz + 1)
    grid = [[v(float(x), 0.0, float(z)) for x in xs] for z in zs]
    for j in range(nz):
        for i in range(nx):
            a, b, c, d = grid[j][i], grid[j][i + 1], grid[j + 1][i + 1], grid[j + 1][i]
            faces_floor += [(a, c, b), (a, d, c)]
    for xw, eps in ((-3.0, 1e-4), (3.0, -1e-4)):         # mirror walls, slightly non-parallel
        a = v(xw, 0.0, -15.0); b = v(xw + eps, 0.0, 0.0); c = v(xw + eps, 2.5, 0.0); d = v(xw, 2.5, -15.0)
        faces_wall += [(a, b, c), (a, c, d)]
    for _ in range(24):                                     # small tiles tilted a hair off the floor
        x, z = rng.uniform(-2.5, 2.5), rng.uniform(-14, -1)
        h = float(rng.uniform(1e-5, 1e-3))
        a = v(x, 0.0, z); b = v(x + 0.4, h, z); c = v(x + 0.4, h, z + 0.4); d = v(x, 0.0, z + 0.4)
        faces_tilt += [(a, b, c), (a, c, d)]
    ctr = v(0.7, 0.3, -6.0)
    cam = (0.0, cam_h, 0.4)
    light = (0.0, 4.0, -4.0)

    def faces(fs):
        return "\n".join(f"                {a} {b} {c}" for a, b, c in fs)

    vd = "\n".join(f"        {_fmt(x)} {_fmt(y)} {_fmt(z)}" for x, y, z in verts)
    w, h = res
    aspect = h / w
    return f"""<Scene>
    <BackgroundColor>20 40 90</BackgroundColor>
    <ShadowRayEpsilon>1e-3</ShadowRayEpsilon>
    <MaxRecursionDepth>{depth}</MaxRecursionDepth>
    <Cameras>
        <Camera id="1">
            <Position>{cam[0]} {cam[1]} {cam[2]}</Position>
            <Gaze>0 -0.0015 -1</Gaze>
            <Up>0 1 0</Up>
            <NearPlane>-0.6 0.6 {-0.6 * aspect:.6f} {0.6 * aspect:.6f}</NearPlane>
            <NearDistance>1</NearDistance>
            <ImageResolution>{w} {h}</ImageResolution>
            <ImageName>grazing.ppm</ImageName>
        </Camera>
    </Cameras>
    <Lights>
        <AmbientLight>20 20 20</AmbientLight>
        <PointLight id="1">
            <Position>{light[0]} {light[1]} {light[2]}</Position>
            <Intensity>900 900 900</Intensity>
        </PointLight>
        <PointLight id="2">
            <Position>-2 0.05 -1</Position>
            <Intensity>40 30 20</Intensity>
        </PointLight>
    </Lights>
    <Materials>
        <Material id="1" type="mirror">
            <AmbientReflectance>0.2 0.2 0.2</AmbientReflectance>
            <DiffuseReflectance>0.3 0.3 0.3</DiffuseReflectance>
            <SpecularReflectance>0.5 0.5 0.5</SpecularReflectance>
            <MirrorReflectance>0.6 0.6 0.6</MirrorReflectance>
            <PhongExponent>50</PhongExponent>
        </Material>
        <Material id="2" type="mirror">
            <AmbientReflectance>0.1 0.1 0.1</AmbientReflectance>
            <DiffuseReflectance>0.1 0.5 0.1</DiffuseReflectance>
            <SpecularReflectance>0.5 0.5 0.5</SpecularReflectance>
            <MirrorReflectance>0.9 0.9 0.9</MirrorReflectance>
            <PhongExponent>3</PhongExponent>
        </Material>
        <Material id="3">
            <AmbientReflectance>0.3 0.1 0.1</AmbientReflectance>
            <DiffuseReflectance>0.8 0.2 0.2</DiffuseReflectance>
            <SpecularReflectance>0.2 0.2 0.2</SpecularReflectance>
            <MirrorReflectance>0 0 0</MirrorReflectance>
            <PhongExponent>1</PhongExponent>
        </Material>
    </Materials>
    <VertexData>
{vd}
    </VertexData>
    <Objects>
        <Mesh id="1">
            <Material>1</Material>
            <Faces>
{faces(faces_floor)}
            </Faces>
        </Mesh>
        <Mesh id="2">
            <Material>2</Material>
            <Faces>
{faces(faces_wall)}
            </Faces>
        </Mesh>
        <Mesh id="3">
            <Material>3</Material>
            <Faces>
{faces(faces_tilt)}
            </Faces>
        </Mesh>
        <Sphere id="1">
            <Material>2</Material>
            <Center>{ctr}</Center>
            <Radius>0.3</Radius>
        </Sphere>
    </Objects>
</Scene>
"""


@pytest.mark.parametrize("wide", ["1", "0"])
@pytest.mark.parametrize("cam_h", [0.02, 1e-3])
def test_grazing_scene_vs_oracle(cam_h, wide, pkg, oracle, tmp_path, torch_cuda, monkeypatch):
    """Whole image and exact work counters against the C oracle, with the wide reference-order walk
    (RT_WIDE_WALK=1, the default) and with the binary reference-tree walk (RT_WIDE_WALK=0)."""
    monkeypatch.setenv("RT_WIDE_WALK", wide)
    p = tmp_path / "grazing.xml"
    p.write_text(grazing_scene(cam_h=cam_h))
    ref, rc = oracle.OracleScene(p).render(0, aa=1)
    with pkg.Scene.from_xml(p, device=0) as s:
        img, st = s.render(s.camera(0), aa=1, stats=True)
        img2, _ = s.render(s.camera(0), aa=1)
    assert np.array_equal(img, ref), f"{int((img != ref).any(axis=2).sum())} pixels differ"
    assert np.array_equal(img2, ref)
    for k in ("primary_rays", "shadow_rays", "reflection_rays", "node_visits", "tri_tests", "sphere_tests"):
        assert st[k] == rc[k], k


def _grazing_rays(rng, n: int) -> np.ndarray:
    """Rays over/along the floor: origins on, just above or below the plane y = 0, directions within a
    few 1e-4 rad of horizontal, plus rays between the mirror walls at grazing angles."""
    o = np.empty((n, 3), np.float32)
    d = np.empty((n, 3), np.float32)
    o[:, 0] = rng.uniform(-7.5, 7.5, n)
    o[:, 2] = rng.uniform(-15.5, 0.3, n)
    kind = rng.integers(0, 4, n)
    o[:, 1] = np.where(kind == 0, 0.0, np.where(kind == 1, 1e-3, np.where(kind == 2, -1e-6, 0.05)))
    ang = rng.uniform(0, 2 * np.pi, n)
    slope = rng.choice([0.0, 1e-6, -1e-6, 3e-4, -3e-4, -2e-3], n)
    d[:, 0] = np.cos(ang)
    d[:, 2] = np.sin(ang)
    d[:, 1] = slope
    # a quarter: near the walls, almost parallel to them
    m = rng.random(n) < 0.25
    o[m, 0] = rng.choice([-2.999, 2.999, -3.0, 3.0], int(m.sum()))
    d[m, 0] = rng.uniform(-1e-4, 1e-4, int(m.sum()))
    d[m, 2] = -1.0
    scale = rng.uniform(0.5, 3.0, n).astype(np.float32)[:, None]     # un-normalised directions (Ray::Ray)
    return np.concatenate([o, d * scale], axis=1).astype(np.float32)


def test_random_grazing_rays_match_reference_walk(pkg, tmp_path, torch_cuda):
    """Closest hit of 60 000 grazing rays: the production walk (rt_walk_timing mode 0, the 4-wide
    reference-order walk) returns the same primitive as the reference's ordered DFS over its binary
    tree (mode 1) for every ray."""
    p = tmp_path / "grazing.xml"
    p.write_text(grazing_scene(nx=64, nz=64))
    rays = _grazing_rays(np.random.default_rng(11), 60000)
    with pkg.Scene.from_xml(p, device=0) as s:
        a = s.walk_timing(rays, lanes=1, reps=1, mode=0)
        b = s.walk_timing(rays, lanes=1, reps=1, mode=1)
        s.check()
    pa, pb = a[:, 2].astype(np.int64), b[:, 2].astype(np.int64)
    assert (pb >= 0).sum() > 10000          # most rays hit something
    bad = np.nonzero(pa != pb)[0]
    assert bad.size == 0, f"{bad.size} rays differ, first {rays[bad[:3]]}"


def test_random_rays_horse_and_mug(pkg, scene_dir, torch_cuda):
    """The same on horse_and_mug (the headline scene): 40 000 rays from random points inside the scene
    box in random directions."""
    from conftest import config_path
    rng = np.random.default_rng(5)
    n = 40000
    o = np.stack([rng.uniform(-17, 17, n), rng.uniform(0.0, 2.7, n), rng.uniform(-18, 16, n)], 1)
    d = rng.normal(size=(n, 3))
    d[rng.random(n) < 0.3, 1] *= 1e-4                      # a third nearly horizontal
    rays = np.concatenate([o, d], 1).astype(np.float32)
    with pkg.Scene.from_xml(config_path(scene_dir, "C3_hm_1080p_d6"), device=0) as s:
        a = s.walk_timing(rays, lanes=1, reps=1, mode=0)
        b = s.walk_timing(rays, lanes=1, reps=1, mode=1)
    assert np.array_equal(a[:, 2], b[:, 2])


def test_walk_step_bound_reports_limit(pkg, scene_dir, torch_cuda, monkeypatch):
    """The always-on walk step bound (traverse2.hpp walk_runaway), forced low: the render ends and the
    call returns RT_ERR_LIMIT instead of running on; a scene with the default bound renders normally."""
    from conftest import config_path
    xml = config_path(scene_dir, "hm_verbatim")
    monkeypatch.setenv("RT_WALK_CAP", "3")
    with pkg.Scene.from_xml(xml, device=0) as s:
        with pytest.raises(pkg.RtError) as ei:
            s.render(s.camera(0), aa=1)
        assert ei.value.code == -6
        assert "step bound" in str(ei.value)
        s.check()                                  # the error word was cleared by the failing call
    monkeypatch.delenv("RT_WALK_CAP")
    with pkg.Scene.from_xml(xml, device=0) as s:
        s.render(s.camera(0), aa=1)
        s.check()


def test_wait_bound_reports_limit(pkg, scene_dir, goldens, torch_cuda, monkeypatch):
    """The always-on bound on the loops that wait on other lanes or waves (pathchain.hip spin_over: the
    phase-A unit hand-off, the phase-B LDS shadow queue, the wave leaf queue), forced to 0: every wait
    gives up at once, so a lone C3 frame (whose phase-B waves wait on the workgroup's shadow queue) ends
    with RT_ERR_LIMIT instead of hanging; with the default bound the same scene renders the golden."""
    from conftest import config_path, golden_by_name, load_golden_image
    g = golden_by_name(goldens, "C3_hm_1080p_d6_aa1")
    xml = config_path(scene_dir, g["config"])
    monkeypatch.setenv("RT_SPIN_CAP", "0")
    with pkg.Scene.from_xml(xml, device=0) as s:
        with pytest.raises(pkg.RtError) as ei:
            s.render(s.camera(0), aa=1)
        assert ei.value.code == -6
        assert "spin_cap" in str(ei.value)
        s.check()                                  # the error word was cleared by the failing call
    monkeypatch.delenv("RT_SPIN_CAP")
    with pkg.Scene.from_xml(xml, device=0) as s:
        img, _ = s.render(s.camera(0), aa=1)
        s.check()
    assert np.array_equal(img, load_golden_image(g["cameras"][0]))


@pytest.mark.parametrize("hot", ["1", "0"])
def test_repeated_lone_frames_equal_golden(pkg, scene_dir, goldens, torch_cuda, monkeypatch, hot):
    """Lone frames deal their phase-A units in the order the previous frame ranked them (rt_api.cpp
    hot_units, pathchain.hip rank_units: the units whose samples walked the most steps first).  Frames of
    one geometry in a row, another geometry between them (the ranking's key changes) and back: every
    frame is the golden."""
    from conftest import config_path, golden_by_name, load_golden_image
    monkeypatch.setenv("RT_HOT_UNITS", hot)
    g1 = golden_by_name(goldens, "C3_hm_1080p_d6_aa1")
    g2 = golden_by_name(goldens, "C3_hm_1080p_d6_aa2")
    ref1, ref2 = load_golden_image(g1["cameras"][0]), load_golden_image(g2["cameras"][0])
    with pkg.Scene.from_xml(config_path(scene_dir, g1["config"]), device=0) as s:
        cam = s.camera(0)
        for aa, ref in ((1, ref1), (1, ref1), (1, ref1), (2, ref2), (1, ref1), (1, ref1)):
            img, _ = s.render(cam, aa=aa)
            assert np.array_equal(img, ref)
        s.check()
