"""Scene fixtures and the derived benchmark scenes.

The reference ships its scenes as XML (`inputs/*.xml`); copies live gzip'd in
tests/golden/scenes/.  BASELINE.json's configs are *derived* from them by
editing the XML text only (so both the reference harness and this framework's
loader parse exactly the same bytes):

  C1  simple.xml verbatim
  C2  cornellbox.xml, only <Camera id="2"> (800x800), MaxRecursionDepth 0
  C3  horse_and_mug.xml, 1920x1080, NearPlane -1 1 -0.5625 0.5625, depth 6
  C5  C3 at 7680x4320 (rendered with SSAA factor 4 = 16 spp)
"""
from __future__ import annotations

import gzip
import os
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SCENE_DIR = ROOT / "tests" / "golden" / "scenes"


def scene_text(name: str) -> str:
    """Text of a reference scene (e.g. 'horse_and_mug.xml')."""
    with gzip.open(SCENE_DIR / (name + ".gz"), "rt") as f:
        return f.read()


def _sub(tag: str, value: str, text: str) -> str:
    pat = re.compile(r"(<%s>)(.*?)(</%s>)" % (tag, tag), re.S)
    out, n = pat.subn(lambda m: m.group(1) + value + m.group(3), text)
    if n == 0:
        raise ValueError(f"tag <{tag}> not found")
    return out


def derive_xml(text: str, depth: int | None = None, res: tuple[int, int] | None = None,
               near: tuple[float, float, float, float] | None = None,
               keep_camera: str | None = None, image_name: str | None = None) -> str:
    """Apply the §8d edits to a scene's XML text."""
    if keep_camera is not None:
        cams = re.compile(r"\s*<Camera id=\"([^\"]*)\">.*?</Camera>", re.S)
        text = cams.sub(lambda m: m.group(0) if m.group(1) == keep_camera else "", text)
    if depth is not None:
        text = _sub("MaxRecursionDepth", str(depth), text)
    if res is not None:
        text = _sub("ImageResolution", f"{res[0]} {res[1]}", text)
    if near is not None:
        text = _sub("NearPlane", " ".join(_fmt(v) for v in near), text)
    if image_name is not None:
        text = _sub("ImageName", image_name, text)
    return text


def _fmt(v: float) -> str:
    return repr(float(v)) if float(v) != int(v) else str(int(v))


# name -> (scene file, derive kwargs)
CONFIGS: dict[str, tuple[str, dict]] = {
    "C1_simple": ("simple.xml", {}),
    "C2_cornellbox_800_d0": ("cornellbox.xml", dict(keep_camera="2", depth=0,
                                                     image_name="cornellbox_800_d0.ppm")),
    "hm_verbatim": ("horse_and_mug.xml", {}),
    "C3_hm_1080p_d6": ("horse_and_mug.xml", dict(depth=6, res=(1920, 1080),
                                                 near=(-1, 1, -0.5625, 0.5625),
                                                 image_name="horse_and_mug_1080p_d6.ppm")),
    "C5_hm_8k_d6": ("horse_and_mug.xml", dict(depth=6, res=(7680, 4320),
                                              near=(-1, 1, -0.5625, 0.5625),
                                              image_name="horse_and_mug_8k_d6.ppm")),
    # timing probe for k_fallback (not a §8d config): an axis-aligned camera at an odd resolution, whose
    # centre column and row have eye-ray direction components of exactly 0 (deferred by the timed walks)
    "X_cornell_801_axis": ("cornellbox.xml", dict(keep_camera="1", res=(801, 801),
                                                   image_name="cornellbox_801_axis.ppm")),
}


def config_xml(name: str) -> str:
    """XML text of a named config: a §8d derived scene or any reference scene file."""
    if name in CONFIGS:
        scene, kw = CONFIGS[name]
        return derive_xml(scene_text(scene), **kw)
    return scene_text(name if name.endswith(".xml") else name + ".xml")


def _strtof():
    """libc strtof: the reference reads its floats with `istream >> float` (parser.cpp), i.e. strtof
    semantics; a Python float rounded to f32 would round twice."""
    import ctypes
    libc = ctypes.CDLL(None)
    f = libc.strtof
    f.restype = ctypes.c_float
    f.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    return lambda tok: f(tok.encode(), None)


def scene_arrays(text: str) -> dict:
    """A scene's XML as the plain arrays of rt_scene_desc (include/rt/rt.h), read the way
    Scene::loadFromXml reads them (parser.cpp:6-218: defaults bg 0 0 0, eps 0.001, depth 0; ids are
    1-based and implicit by order; `type="mirror"` sets is_mirror), with the triangles in the
    RayTracer ctor's flattening order (raytracer.cpp:336-341): the standalone <Triangle>s, then each
    <Mesh>'s faces with the mesh's material.  Cameras are returned beside them (rt_camera fields)."""
    import xml.etree.ElementTree as ET
    sf = _strtof()
    root = ET.fromstring(text)

    def floats(t):
        return [sf(v) for v in t.split()]

    def ints(t):
        return [int(v) for v in t.split()]

    def opt(tag, default):
        e = root.find(tag)
        return e.text if e is not None else default

    lights_el = root.find("Lights")
    out = {
        "background_color": ints(opt("BackgroundColor", "0 0 0"))[:3],
        "shadow_ray_epsilon": floats(opt("ShadowRayEpsilon", "0.001"))[0],
        "max_recursion_depth": ints(opt("MaxRecursionDepth", "0"))[0],
        "ambient_light": floats(lights_el.find("AmbientLight").text)[:3],
        "lights": [(floats(pl.find("Position").text)[:3], floats(pl.find("Intensity").text)[:3])
                   for pl in lights_el.findall("PointLight")],
        "materials": [dict(is_mirror=1 if m.get("type") == "mirror" else 0,
                           ambient=floats(m.find("AmbientReflectance").text)[:3],
                           diffuse=floats(m.find("DiffuseReflectance").text)[:3],
                           specular=floats(m.find("SpecularReflectance").text)[:3],
                           mirror=floats(m.find("MirrorReflectance").text)[:3],
                           phong_exponent=floats(m.find("PhongExponent").text)[0])
                      for m in root.find("Materials").findall("Material")],
    }
    vd = floats(root.find("VertexData").text)
    out["vertices"] = [vd[i:i + 3] for i in range(0, len(vd) - len(vd) % 3, 3)]
    objs = root.find("Objects")
    tris = [(int(t.find("Material").text), *ints(t.find("Indices").text)[:3]) for t in objs.findall("Triangle")]
    for m in objs.findall("Mesh"):
        mid = int(m.find("Material").text)
        f = ints(m.find("Faces").text)
        tris += [(mid, f[i], f[i + 1], f[i + 2]) for i in range(0, len(f) - len(f) % 3, 3)]
    out["triangles"] = tris
    out["spheres"] = [(int(s.find("Material").text), int(s.find("Center").text), sf(s.find("Radius").text.strip()))
                      for s in objs.findall("Sphere")]
    cams = []
    for c in root.find("Cameras").findall("Camera"):
        res = ints(c.find("ImageResolution").text)
        cams.append(dict(position=floats(c.find("Position").text)[:3], gaze=floats(c.find("Gaze").text)[:3],
                         up=floats(c.find("Up").text)[:3], near_plane=floats(c.find("NearPlane").text)[:4],
                         near_distance=floats(c.find("NearDistance").text)[0], image_width=res[0],
                         image_height=res[1], image_name=c.find("ImageName").text.strip()))
    out["cameras"] = cams
    return out


def write_config(name: str, directory: str | os.PathLike) -> str:
    """Write the config's XML into `directory`; return its path."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    p = d / (name if name.endswith(".xml") else name + ".xml")
    p.write_text(config_xml(name))
    return str(p)
