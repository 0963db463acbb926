"""Python view of librt_hip.so (the MI355X-native renderer) through its C-ABI.

The product is the C-ABI library (include/rt/rt.h) and the drop-in C++ CLI
(`raytracer scene.xml`, raytracer.cpp:487-525 semantics).  This module is the
thin ctypes layer the tests and bench.py use: scene load, render into host or
device (HBM) buffers, stripe helpers for the multi-GPU path, write_ppm.

There is no CPU fallback: if librt_hip.so is missing this module raises on
import of the library, and rendering requires a visible gfx950 device.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

import numpy as np

from . import scenes  # noqa: F401  (re-export: scene fixtures / derived configs)
from . import stripes  # noqa: F401
from . import frame  # noqa: F401  (multi-GPU slab gather + reassembly)

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["RT_LIB"]) if os.environ.get("RT_LIB") else PKG_DIR / "librt_hip.so"   # RT_LIB: experiments
CLI_PATH = PKG_DIR / "raytracer"

RT_OPT_HOST_ONLY = 1
RT_OPT_CHAIN = 8
PATHS = ("chain",)        # the one render path (rt.h: the comparison paths were removed in ABI 11)
RT_RENDER_COUNT = 1


class RtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rt error {code}: {msg}")
        self.code = code


class Vec3f(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float)]


class Camera(ctypes.Structure):
    """rt_camera == parser::Camera (parser.h:170-178) minus image_name."""
    _fields_ = [("position", Vec3f), ("gaze", Vec3f), ("up", Vec3f),
                ("near_plane", ctypes.c_float * 4), ("near_distance", ctypes.c_float),
                ("image_width", ctypes.c_int), ("image_height", ctypes.c_int)]


class Options(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("flags", ctypes.c_int), ("build_threads", ctypes.c_int)]


class Stats(ctypes.Structure):
    _fields_ = [("primary_rays", ctypes.c_uint64), ("shadow_rays", ctypes.c_uint64),
                ("reflection_rays", ctypes.c_uint64), ("node_visits", ctypes.c_uint64),
                ("tri_tests", ctypes.c_uint64), ("sphere_tests", ctypes.c_uint64),
                ("kernel_ms", ctypes.c_double), ("wall_ms", ctypes.c_double),
                ("shadow_rays_skipped", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class BvhInfo(ctypes.Structure):
    _fields_ = [("nodes", ctypes.c_int), ("leaves", ctypes.c_int), ("max_leaf_prims", ctypes.c_int),
                ("max_depth", ctypes.c_int), ("max_stack", ctypes.c_int), ("triangles", ctypes.c_int),
                ("spheres", ctypes.c_int), ("build_ms", ctypes.c_double),
                ("ref_ms", ctypes.c_double), ("wide_ms", ctypes.c_double), ("build_threads", ctypes.c_int),
                ("wide_nodes", ctypes.c_int), ("wide_hash", ctypes.c_uint64),
                ("ref_wide_bytes", ctypes.c_uint64), ("occ_wide_bytes", ctypes.c_uint64),
                ("leaf_record_bytes", ctypes.c_uint64), ("tri_shade_bytes", ctypes.c_uint64),
                ("xml_ms", ctypes.c_double), ("prep_ms", ctypes.c_double), ("flat_ms", ctypes.c_double),
                ("refwide_ms", ctypes.c_double), ("stree_ms", ctypes.c_double), ("upload_ms", ctypes.c_double)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class PointLight(ctypes.Structure):     # rt_point_light (parser.h:180-183)
    _fields_ = [("position", Vec3f), ("intensity", Vec3f)]


class Material(ctypes.Structure):       # rt_material (parser.h:185-192)
    _fields_ = [("is_mirror", ctypes.c_int), ("ambient", Vec3f), ("diffuse", Vec3f), ("specular", Vec3f),
                ("mirror", Vec3f), ("phong_exponent", ctypes.c_float)]


class Triangle(ctypes.Structure):       # rt_triangle: material id, 1-based vertex ids
    _fields_ = [("material_id", ctypes.c_int), ("v0_id", ctypes.c_int), ("v1_id", ctypes.c_int),
                ("v2_id", ctypes.c_int)]


class Sphere(ctypes.Structure):         # rt_sphere
    _fields_ = [("material_id", ctypes.c_int), ("center_vertex_id", ctypes.c_int), ("radius", ctypes.c_float)]


class SceneDesc(ctypes.Structure):      # rt_scene_desc: borrowed host arrays
    _fields_ = [("background_color", ctypes.c_int * 3), ("shadow_ray_epsilon", ctypes.c_float),
                ("max_recursion_depth", ctypes.c_int), ("ambient_light", Vec3f),
                ("lights", ctypes.POINTER(PointLight)), ("num_lights", ctypes.c_int),
                ("materials", ctypes.POINTER(Material)), ("num_materials", ctypes.c_int),
                ("vertices", ctypes.POINTER(Vec3f)), ("num_vertices", ctypes.c_int),
                ("triangles", ctypes.POINTER(Triangle)), ("num_triangles", ctypes.c_int),
                ("spheres", ctypes.POINTER(Sphere)), ("num_spheres", ctypes.c_int)]


def make_desc(a: dict) -> tuple[SceneDesc, list]:
    """rt_scene_desc over ctypes arrays built from scenes.scene_arrays(); returns (desc, keepalive)."""
    def v3(x):
        return Vec3f(*x)

    def arr(T, xs):
        return (T * max(1, len(xs)))(*xs)

    lights = arr(PointLight, [PointLight(v3(p), v3(i)) for p, i in a["lights"]])
    mats = arr(Material, [Material(m["is_mirror"], v3(m["ambient"]), v3(m["diffuse"]), v3(m["specular"]),
                                   v3(m["mirror"]), m["phong_exponent"]) for m in a["materials"]])
    verts = arr(Vec3f, [v3(v) for v in a["vertices"]])
    tris = arr(Triangle, [Triangle(*t) for t in a["triangles"]])
    sph = arr(Sphere, [Sphere(*s) for s in a["spheres"]])
    d = SceneDesc((ctypes.c_int * 3)(*a["background_color"]), a["shadow_ray_epsilon"], a["max_recursion_depth"],
                  v3(a["ambient_light"]), lights, len(a["lights"]), mats, len(a["materials"]), verts,
                  len(a["vertices"]), tris, len(a["triangles"]), sph, len(a["spheres"]))
    return d, [lights, mats, verts, tris, sph]


def camera_from(c: dict) -> "Camera":
    """rt_camera from a scenes.scene_arrays() camera entry."""
    return Camera(Vec3f(*c["position"]), Vec3f(*c["gaze"]), Vec3f(*c["up"]), (ctypes.c_float * 4)(*c["near_plane"]),
                  c["near_distance"], c["image_width"], c["image_height"])


# device_layout.hpp dl::Node (32 B)
NODE_DTYPE = np.dtype([("minx", "<f4"), ("miny", "<f4"), ("minz", "<f4"), ("a", "<i4"),
                       ("maxx", "<f4"), ("maxy", "<f4"), ("maxz", "<f4"), ("b", "<i4")])

# (name, restype, argtypes) for every function declared in include/rt/rt.h
_P = ctypes.c_void_p
_SIGS = [
    ("rt_last_error", ctypes.c_char_p, []),
    ("rt_abi_version", ctypes.c_int, []),
    ("rt_device_count", ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    ("rt_set_devices", ctypes.c_int, [ctypes.c_int]),
    ("rt_scene_num_devices", ctypes.c_int, [_P]),
    ("rt_scene_create", ctypes.c_int, [_P, ctypes.POINTER(Options), ctypes.POINTER(_P)]),
    ("rt_scene_load_xml", ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(Options), ctypes.POINTER(_P)]),
    ("rt_scene_destroy", None, [_P]),
    ("rt_scene_num_cameras", ctypes.c_int, [_P]),
    ("rt_scene_get_camera", ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(Camera), ctypes.c_char_p, ctypes.c_int]),
    ("rt_scene_bvh_info", ctypes.c_int, [_P, ctypes.POINTER(BvhInfo)]),
    ("rt_scene_set_max_depth", ctypes.c_int, [_P, ctypes.c_int]),
    ("rt_scene_export_nodes", ctypes.c_int, [_P, _P, ctypes.c_int]),
    ("rt_render", ctypes.c_int, [_P, ctypes.POINTER(Camera), ctypes.c_int, _P, ctypes.POINTER(Stats)]),
    ("rt_render_device", ctypes.c_int, [_P, ctypes.POINTER(Camera), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, _P, _P, ctypes.c_int]),
    ("rt_render_cameras", ctypes.c_int, [_P, ctypes.POINTER(Camera), ctypes.c_int, ctypes.c_int, _P,
                                         ctypes.POINTER(Stats)]),
    ("rt_render_cameras_device", ctypes.c_int, [_P, ctypes.POINTER(Camera), ctypes.c_int, ctypes.c_int, _P, _P,
                                                ctypes.c_int]),
    ("rt_render_frames_device", ctypes.c_int, [_P, ctypes.POINTER(Camera), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, _P, _P, ctypes.c_int]),
    ("rt_walk_timing", ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P]),
    ("rt_phong_pow", ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    ("rt_cramer_div", ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    ("rt_udiv", ctypes.c_int, [_P, ctypes.c_int, _P, ctypes.c_int, _P]),
    ("rt_measure_peaks", ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, _P]),
    ("rt_scene_memory", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    ("rt_slab_rows", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    ("rt_unshuffle_stripes", ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P]),
    ("rt_counters_reset", ctypes.c_int, [_P, _P]),
    ("rt_counters_read", ctypes.c_int, [_P, ctypes.POINTER(Stats)]),
    ("rt_counters_read_raw", ctypes.c_int, [_P, _P, ctypes.c_int]),
    ("rt_kernel_times", ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int]),
    ("rt_scene_check", ctypes.c_int, [_P]),
    ("rt_primary_hits", ctypes.c_int, [_P, ctypes.POINTER(Camera), ctypes.c_int, _P, _P]),
    ("rt_primary_hits_production", ctypes.c_int, [_P, ctypes.POINTER(Camera), ctypes.c_int, _P, _P]),
    ("rt_downsample_host", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P]),
    ("rt_write_ppm", ctypes.c_int, [ctypes.c_char_p, _P, ctypes.c_int, ctypes.c_int]),
]

_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """Load librt_hip.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RtError(-5, f"{LIB_PATH} not built (run __graft_entry__.build())")
        L = ctypes.CDLL(str(LIB_PATH))
        for name, res, args in _SIGS:
            if os.environ.get("RT_LIB") and not hasattr(L, name):
                continue          # an older experiment build (RT_LIB) may lack newer entry points
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != 0:
        raise RtError(rc, lib().rt_last_error().decode())


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(lib().rt_device_count(ctypes.byref(n)))
    return n.value


def set_devices(n: int) -> None:
    """rt_set_devices: scenes created afterwards render every frame on GPUs 0..n-1 (row stripes, one
    RCCL gather to device 0); 1 = the same group path on one GPU; 0 = no group (default)."""
    _check(lib().rt_set_devices(n))


def phong_pow(base, exponent) -> np.ndarray:
    """Diagnostics (rt_phong_pow): the device's specular power term,
    (float)pow((double)base, (double)exponent) as raytracer.cpp:414 computes it."""
    b = np.ascontiguousarray(base, dtype=np.float32)
    e = np.ascontiguousarray(exponent, dtype=np.float32)
    if b.shape != e.shape:
        raise ValueError("base and exponent differ in shape")
    out = np.empty_like(b)
    _check(lib().rt_phong_pow(b.ctypes.data_as(ctypes.c_void_p), e.ctypes.data_as(ctypes.c_void_p),
                              out.ctypes.data_as(ctypes.c_void_p), b.size))
    return out


def cramer_div(den, num) -> np.ndarray:
    """Diagnostics (rt_cramer_div): num[i, j] / den[i] (j = 0..2) as the device's triangle test
    computes its Cramer quotients (raytracer.cpp:147, 154, 161)."""
    d = np.ascontiguousarray(den, dtype=np.float32).reshape(-1)
    nm = np.ascontiguousarray(num, dtype=np.float32).reshape(-1, 3)
    if nm.shape[0] != d.size:
        raise ValueError("num must hold three numerators per denominator")
    out = np.empty_like(nm)
    _check(lib().rt_cramer_div(d.ctypes.data_as(ctypes.c_void_p), nm.ctypes.data_as(ctypes.c_void_p),
                               out.ctypes.data_as(ctypes.c_void_p), d.size))
    return out


def udiv(v, d) -> np.ndarray:
    """Diagnostics (rt_udiv): v[i] // d[j] as the shadow walkers divide by a wave-uniform divisor
    (pathchain.hip UDiv); returns shape (len(d), len(v)), uint32."""
    vv = np.ascontiguousarray(v, dtype=np.uint32).reshape(-1)
    dd = np.ascontiguousarray(d, dtype=np.uint32).reshape(-1)
    q = np.empty((dd.size, vv.size), dtype=np.uint32)
    _check(lib().rt_udiv(vv.ctypes.data_as(ctypes.c_void_p), vv.size, dd.ctypes.data_as(ctypes.c_void_p), dd.size,
                         q.ctypes.data_as(ctypes.c_void_p)))
    return q


class Peaks(ctypes.Structure):
    _fields_ = [("hbm_copy_gbps", ctypes.c_double), ("hbm_read_gbps", ctypes.c_double),
                ("l2_gather_gbps", ctypes.c_double), ("l2_table_bytes", ctypes.c_double),
                ("scene_gather_gbps", ctypes.c_double), ("scene_table_bytes", ctypes.c_double),
                ("l2_line_gbps", ctypes.c_double), ("scene_line_gbps", ctypes.c_double)]


def measure_peaks(device: int = -1, scene_table_bytes: int = 6 << 20) -> dict:
    """rt_measure_peaks: measured HBM copy/read and walk-shaped L2 gather bandwidths (GB/s)."""
    p = Peaks()
    _check(lib().rt_measure_peaks(device, scene_table_bytes, ctypes.byref(p)))
    return {k: getattr(p, k) for k, _ in p._fields_}


def slab_rows(height: int, stripe_rows: int, nranks: int) -> int:
    return lib().rt_slab_rows(height, stripe_rows, nranks)


class Scene:
    """An rt_scene: host scene + bit-exact BVH + device copies (one GPU)."""

    def __init__(self, handle: int):
        self._h = ctypes.c_void_p(handle)

    @classmethod
    def from_xml(cls, path: str | os.PathLike, device: int = -1, host_only: bool = False,
                 render_path: str = "chain", build_threads: int = 0) -> "Scene":
        """render_path: "chain" or "default" (the same: the library has one render path).
        build_threads: host BVH build threads (0: default, 1: serial); the tree does not depend on it."""
        h = ctypes.c_void_p()
        flags = RT_OPT_HOST_ONLY if host_only else 0
        flags |= {"chain": RT_OPT_CHAIN, "default": 0}[render_path]
        opts = Options(device, flags, build_threads)
        _check(lib().rt_scene_load_xml(str(path).encode(), ctypes.byref(opts), ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def from_desc(cls, arrays: dict, device: int = -1, host_only: bool = False,
                  render_path: str = "chain") -> "Scene":
        """rt_scene_create from borrowed host arrays (the reference's RayTracer(parser::Scene&) ctor,
        raytracer.cpp:335-350); `arrays` as returned by scenes.scene_arrays()."""
        desc, keep = make_desc(arrays)
        h = ctypes.c_void_p()
        flags = RT_OPT_HOST_ONLY if host_only else 0
        flags |= {"chain": RT_OPT_CHAIN, "default": 0}[render_path]
        opts = Options(device, flags, 0)
        _check(lib().rt_scene_create(ctypes.byref(desc), ctypes.byref(opts), ctypes.byref(h)))
        del keep
        return cls(h.value)

    def close(self) -> None:
        if self._h and self._h.value:
            lib().rt_scene_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def cameras(self) -> list[tuple[Camera, str]]:
        out = []
        for i in range(lib().rt_scene_num_cameras(self._h)):
            cam = Camera()
            name = ctypes.create_string_buffer(1024)
            _check(lib().rt_scene_get_camera(self._h, i, ctypes.byref(cam), name, 1024))
            out.append((cam, name.value.decode()))
        return out

    def camera(self, index: int = 0) -> Camera:
        return self.cameras()[index][0]

    def bvh_info(self) -> dict:
        info = BvhInfo()
        _check(lib().rt_scene_bvh_info(self._h, ctypes.byref(info)))
        return info.as_dict()

    def export_nodes(self) -> np.ndarray:
        n = lib().rt_scene_export_nodes(self._h, None, 0)
        if n < 0:
            _check(n)
        arr = np.zeros(n, dtype=NODE_DTYPE)
        lib().rt_scene_export_nodes(self._h, arr.ctypes.data_as(ctypes.c_void_p), n)
        return arr

    def set_max_depth(self, depth: int) -> None:
        _check(lib().rt_scene_set_max_depth(self._h, depth))

    def render_cameras(self, cams: list, aa: int = 1, stats: bool = False) -> tuple[list, Optional[dict]]:
        """All cameras in one batched call (rt_render_cameras: frames run concurrently on the GPU);
        returns one (H, W, 3) uint8 array per camera, each identical to render() of that camera."""
        n = len(cams)
        arr = (Camera * n)(*cams)
        imgs = [np.empty((c.image_height, c.image_width, 3), dtype=np.uint8) for c in cams]
        ptrs = (ctypes.c_void_p * n)(*[im.ctypes.data for im in imgs])
        st = Stats() if stats else None
        _check(lib().rt_render_cameras(self._h, arr, n, aa, ptrs, ctypes.byref(st) if st is not None else None))
        return imgs, (st.as_dict() if st is not None else None)

    def render_cameras_device(self, cams: list, aa: int, out_ptrs: list, stream: int = 0, count: bool = False) -> None:
        """Asynchronous batched render into device buffers (rt_render_cameras_device)."""
        n = len(cams)
        arr = (Camera * n)(*cams)
        ptrs = (ctypes.c_void_p * n)(*out_ptrs)
        _check(lib().rt_render_cameras_device(self._h, arr, n, aa, ptrs, ctypes.c_void_p(stream),
                                              RT_RENDER_COUNT if count else 0))

    def render_frames_device(self, cams: list, aa: int, out_ptrs: list, stream: int = 0, stripe_rows: int = 8,
                             rank: int = 0, nranks: int = 1, count: bool = False) -> None:
        """Asynchronous render of this rank's stripes of several frames, in flight together
        (rt_render_frames_device); out_ptrs[i] receives frame i's slab, as render_device would."""
        n = len(cams)
        arr = (Camera * n)(*cams)
        ptrs = (ctypes.c_void_p * n)(*out_ptrs)
        _check(lib().rt_render_frames_device(self._h, arr, n, aa, stripe_rows, rank, nranks, ptrs,
                                             ctypes.c_void_p(stream), RT_RENDER_COUNT if count else 0))

    def walk_timing(self, rays, lanes: int = 1, reps: int = 3, mode: int = 0) -> np.ndarray:
        """Diagnostics (rt_walk_timing): rows {cycles, steps, prim, first-rep cycles} per ray."""
        r = np.ascontiguousarray(np.asarray(rays, dtype=np.float32).reshape(-1, 6))
        out = np.zeros((len(r), 4), dtype=np.uint64)
        _check(lib().rt_walk_timing(self._h, r.ctypes.data_as(ctypes.c_void_p), len(r), lanes, reps, mode,
                                    out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def render(self, cam: Camera, aa: int = 1, stats: bool = False) -> tuple[np.ndarray, Optional[dict]]:
        """Synchronous render to a host (H, W, 3) uint8 array (rt_render)."""
        img = np.empty((cam.image_height, cam.image_width, 3), dtype=np.uint8)
        st = Stats() if stats else None
        _check(lib().rt_render(self._h, ctypes.byref(cam), aa, img.ctypes.data_as(ctypes.c_void_p),
                               ctypes.byref(st) if st is not None else None))
        return img, (st.as_dict() if st is not None else None)

    def render_device(self, cam: Camera, aa: int, out_ptr: int, stream: int = 0, stripe_rows: int | None = None,
                      rank: int = 0, nranks: int = 1, count: bool = False) -> None:
        """Asynchronous render of this rank's stripes into device memory (rt_render_device)."""
        sr = stripe_rows if stripe_rows is not None else cam.image_height
        _check(lib().rt_render_device(self._h, ctypes.byref(cam), aa, sr, rank, nranks, ctypes.c_void_p(out_ptr),
                                      ctypes.c_void_p(stream), RT_RENDER_COUNT if count else 0))

    def counters_reset(self, stream: int = 0) -> None:
        _check(lib().rt_counters_reset(self._h, ctypes.c_void_p(stream)))

    def counters_read(self) -> dict:
        st = Stats()
        _check(lib().rt_counters_read(self._h, ctypes.byref(st)))
        return st.as_dict()

    def memory(self) -> dict:
        """HBM the scene holds (rt_scene_memory): uploaded scene and render workspaces, bytes."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().rt_scene_memory(self._h, ctypes.byref(a), ctypes.byref(b)))
        return {"scene_bytes": a.value, "workspace_bytes": b.value}

    COUNTER_SLOTS = ("a_walk_bytes", "a_walks", "a_hits", "b_walk_bytes", "b_walks", "b_hits", "continuations",
                     "a_shadow_bytes", "a_shadow_rays", "bq_shadow_bytes", "bq_shadow_rays", "bo_shadow_bytes",
                     "bo_shadow_rays")

    def counters_raw(self) -> dict:
        """rt_counters_read_raw: the per-role counter slots (pathchain.hpp CounterSlot) by name."""
        out = np.zeros(32, dtype=np.uint64)
        n = lib().rt_counters_read_raw(self._h, out.ctypes.data_as(ctypes.c_void_p), 32)
        if n < 0:
            _check(n)
        res = {k: int(out[8 + i]) for i, k in enumerate(self.COUNTER_SLOTS)}
        res.update({k: int(out[24 + i]) for i, k in enumerate(self.FALLBACK_SLOTS)})
        return res

    # slots 24.. (pathchain.hpp kCntFb*): per chain launch, what the timed walks left to k_fallback
    FALLBACK_SLOTS = ("fb_launches", "fb_continuations", "fb_continuations_beyond_cb", "fb_deferred_closest",
                      "fb_deferred_shadow", "fb_shadow_queue_overflows", "compact_launches")

    KERNEL_KINDS = ("k_chain", "k_pack_a", "k_mix", "k_occlude_a", "k_pack_b", "k_occlude_b", "k_finish", "k_fallback")

    def kernel_times(self, reset: bool = True) -> tuple[dict, int]:
        """rt_kernel_times (scenes created with RT_DEBUG 0x10): ms per kernel of the chain launches, and the launch count."""
        ms = np.zeros(16, dtype=np.float64)
        n = lib().rt_kernel_times(self._h, ms.ctypes.data_as(ctypes.c_void_p), 16, int(reset))
        if n < 0:
            _check(n)
        return {k: float(ms[i]) for i, k in enumerate(self.KERNEL_KINDS)}, n

    def num_devices(self) -> int:
        return lib().rt_scene_num_devices(self._h)

    def check(self) -> None:
        """Synchronise and raise RtError(RT_ERR_LIMIT) if a walk was cut off by its step bound since the
        last check (rt_scene_check)."""
        _check(lib().rt_scene_check(self._h))

    def primary_hits(self, cam: Camera, aa: int = 1, walk: str = "reference") -> tuple[np.ndarray, np.ndarray]:
        """Level-0 closest hit per internal pixel: tSmall (-1 on a miss) and material id (0 on a miss).
        walk="production": the timed kernels' own walk (rt_primary_hits_production: k_chain with the two
        stores added, k_fallback for deferred rays); "reference": the side kernel's binary-tree walk
        (rt_primary_hits)."""
        H, W = cam.image_height * aa, cam.image_width * aa
        t = np.empty((H, W), dtype=np.float32)
        m = np.empty((H, W), dtype=np.int32)
        fn = {"reference": lib().rt_primary_hits, "production": lib().rt_primary_hits_production}[walk]
        _check(fn(self._h, ctypes.byref(cam), aa, t.ctypes.data_as(ctypes.c_void_p), m.ctypes.data_as(ctypes.c_void_p)))
        return t, m


def unshuffle_stripes(slabs_ptr: int, image_ptr: int, width: int, height: int, stripe_rows: int, nranks: int,
                      stream: int = 0) -> None:
    _check(lib().rt_unshuffle_stripes(ctypes.c_void_p(slabs_ptr), ctypes.c_void_p(image_ptr), width, height,
                                      stripe_rows, nranks, ctypes.c_void_p(stream)))


def write_ppm(path: str | os.PathLike, img: np.ndarray) -> None:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    _check(lib().rt_write_ppm(str(path).encode(), img.ctypes.data_as(ctypes.c_void_p), w, h))


def downsample_host(img: np.ndarray, factor: int) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    out = np.empty((h // factor, w // factor, 3), dtype=np.uint8)
    _check(lib().rt_downsample_host(img.ctypes.data_as(ctypes.c_void_p), w, h, factor,
                                    out.ctypes.data_as(ctypes.c_void_p)))
    return out
