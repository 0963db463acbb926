"""ORACLE / TEST INFRASTRUCTURE ONLY — ctypes view of oracle/liboracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline, never as the product path.
liboracle.so is the plain-C restatement of the reference (rt_oracle.c), pinned
bit-exact against the compiled reference through tests/golden/.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"
REF_HARNESS = HERE / "_ref" / "ref_harness"


class Counters(ctypes.Structure):
    _fields_ = [("primary_rays", ctypes.c_uint64), ("shadow_rays", ctypes.c_uint64),
                ("reflection_rays", ctypes.c_uint64), ("node_visits", ctypes.c_uint64),
                ("tri_tests", ctypes.c_uint64), ("sphere_tests", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE), "liboracle.so", "rt_oracle_cli"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        P = ctypes.c_void_p
        L.ro_load.restype = P
        L.ro_load.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.ro_free.argtypes = [P]
        L.ro_num_cameras.argtypes = [P]
        L.ro_camera_info.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                     ctypes.c_char_p, ctypes.c_int]
        L.ro_bvh_info.argtypes = [P] + [ctypes.POINTER(ctypes.c_int)] * 5
        L.ro_render.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, P, ctypes.POINTER(Counters)]
        L.ro_primary_hits.argtypes = [P, ctypes.c_int, ctypes.c_int, P, P]
        L.ro_write_ppm.argtypes = [ctypes.c_char_p, P, ctypes.c_int, ctypes.c_int]
        L.ro_export_nodes.argtypes = [P, P, ctypes.c_int]
        L.ro_work_map.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P]
        _lib = L
    return _lib


# rt_oracle.h ro_node_export: matches the product's 32-byte device node layout
NODE_DTYPE = np.dtype([("minx", "<f4"), ("miny", "<f4"), ("minz", "<f4"), ("a", "<i4"),
                       ("maxx", "<f4"), ("maxy", "<f4"), ("maxz", "<f4"), ("b", "<i4")])


class OracleScene:
    def __init__(self, path: str | os.PathLike):
        err = ctypes.create_string_buffer(256)
        self._h = lib().ro_load(str(path).encode(), err, 256)
        if not self._h:
            raise RuntimeError(err.value.decode())

    def close(self):
        if self._h:
            lib().ro_free(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def cameras(self) -> list[tuple[int, int, str]]:
        out = []
        for i in range(lib().ro_num_cameras(self._h)):
            w, h = ctypes.c_int(), ctypes.c_int()
            name = ctypes.create_string_buffer(256)
            lib().ro_camera_info(self._h, i, ctypes.byref(w), ctypes.byref(h), name, 256)
            out.append((w.value, h.value, name.value.decode()))
        return out

    def bvh_info(self) -> dict:
        v = [ctypes.c_int() for _ in range(5)]
        lib().ro_bvh_info(self._h, *[ctypes.byref(x) for x in v])
        return dict(zip(["nodes", "leaves", "max_leaf", "triangles", "spheres"], [x.value for x in v]))

    def export_nodes(self) -> np.ndarray:
        n = lib().ro_export_nodes(self._h, None, 0)
        arr = np.zeros(n, dtype=NODE_DTYPE)
        lib().ro_export_nodes(self._h, arr.ctypes.data_as(ctypes.c_void_p), n)
        return arr

    def render(self, cam: int = 0, aa: int = 1, threads: int = 0, rows: tuple[int, int] | None = None,
               max_depth: int | None = None) -> tuple[np.ndarray, dict]:
        w, h, _ = self.cameras()[cam]
        r0, r1 = rows if rows is not None else (0, h)
        img = np.zeros((r1 - r0, w, 3), dtype=np.uint8)
        c = Counters()
        t = threads if threads > 0 else (os.cpu_count() or 1)
        rc = lib().ro_render(self._h, cam, aa, t, r0, r1, -1000 if max_depth is None else max_depth,
                             img.ctypes.data_as(ctypes.c_void_p), ctypes.byref(c))
        if rc != 0:
            raise RuntimeError("ro_render failed")
        return img, c.as_dict()

    def primary_hits(self, cam: int = 0, aa: int = 1) -> tuple[np.ndarray, np.ndarray]:
        w, h, _ = self.cameras()[cam]
        t = np.zeros((h * aa, w * aa), dtype=np.float32)
        m = np.zeros((h * aa, w * aa), dtype=np.int32)
        lib().ro_primary_hits(self._h, cam, aa, t.ctypes.data_as(ctypes.c_void_p), m.ctypes.data_as(ctypes.c_void_p))
        return t, m


def write_ppm(path: str | os.PathLike, img: np.ndarray) -> None:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    if lib().ro_write_ppm(str(path).encode(), img.ctypes.data_as(ctypes.c_void_p), img.shape[1], img.shape[0]):
        raise RuntimeError("ro_write_ppm failed")
