"""ctypes binding of the CPU oracle (oracle/oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (as the checker)
and bench.py's cpu_baseline leg (as the timed CPU baseline).  Never the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
EV_NAMES = ("node", "leaf", "prim", "cand", "geom", "colmat", "sample", "trav", "mesh", "tri", "mgeom")
# bytes per event: node 48, leaf 4, prim 16+64, cand 64, geom 64, col+mat 32, sample 24
EV_BYTES = np.array([48, 4, 80, 64, 64, 32, 24, 0, 140, 48, 148], np.int64)

_fp = ctypes.POINTER(ctypes.c_float)
_ip = ctypes.POINTER(ctypes.c_int)
_up = ctypes.POINTER(ctypes.c_uint)
_u64p = ctypes.POINTER(ctypes.c_ulonglong)
_vp = ctypes.c_void_p
_L = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i, f = ctypes.c_int, ctypes.c_float
        sigs = {
            "orc_scene_build": (_vp, [i, f]),
            "orc_scene_free": (None, [_vp]),
            "orc_scene_new": (_vp, [f]),
            "orc_scene_add": (i, [_vp, i, _fp, _fp]),
            "orc_scene_finalize": (i, [_vp]),
            "orc_scene_n_prims": (i, [_vp]),
            "orc_scene_depth": (i, [_vp]),
            "orc_scene_n_emissive": (i, [_vp]),
            "orc_scene_export": (i, [_vp, _fp, _fp, _ip]),
            "orc_camera": (None, [i, i, _fp, _fp]),
            "orc_render": (i, [_fp, i, _fp, _ip, i, _fp, _fp, i, i, i, i, f, i, f, i, i, i, i, _fp, _u64p, _up, _vp]),
            "orc_render_pixels": (i, [_fp, i, _fp, _ip, i, _fp, _fp, i, i, _ip, i, i, i, f, i, f, i, i, i, _fp]),
            "orc_xxhash32": (ctypes.c_uint, [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]),
            "orc_srand": (None, [f, f, i, f, _up]),
            "orc_random_floats": (None, [_up, i, _fp]),
            "orc_sincos": (None, [f, _fp, _fp]),
            "orc_log": (f, [f]),
            "orc_exp2": (f, [f]),
            "orc_pow": (f, [f, f]),
            "orc_random_ray": (None, [_up, _fp, f, _fp, _up]),
            "orc_intersect_prim": (i, [_fp, _fp, _fp, _fp, _ip, _fp, _fp]),
            "orc_corner_rays": (None, [_fp, _fp, _fp]),
            "orc_trace": (i, [_fp, i, _fp, _ip, i, _fp, _fp, i, i, i, _ip, _fp, _vp]),
            "orc_mesh_view": (_vp, [_ip, _fp, _ip, _ip, _fp, _fp, i, i]),
            "orc_mesh_view_free": (None, [_vp]),
            "orc_mesh_bvh": (i, [_fp, _ip, i, _fp, _ip]),
            "orc_sample_hemisphere": (None, [_fp, _fp, f, i, i, _fp]),
            "orc_set_deviation": (i, [i]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _L = L
    return _L


# deviations from the arithmetic contract (oracle.cpp DEV_*): measurement of what the pieces the
# reference leaves to the GL driver / Eigen would change (tests/test_oracle_variants.py only)
DEV_TC_UP, DEV_TC_DOWN, DEV_LIBM, DEV_DIV, DEV_INV_F32 = 1, 2, 4, 8, 16


class deviation:
    """``with deviation(flags): ...`` renders/builds with the given DEV_* flags, then restores."""

    def __init__(self, flags: int):
        self.flags = int(flags)

    def __enter__(self):
        self.old = lib().orc_set_deviation(self.flags)
        return self

    def __exit__(self, *exc):
        lib().orc_set_deviation(self.old)


def P(a: np.ndarray, t=_fp):
    return a.ctypes.data_as(t)


def scene(scene_id: int, light_intensity: float = 1.2) -> Tuple[np.ndarray, np.ndarray, np.ndarray, int, int]:
    """(prims n×64, nodes, leaves, depth, nb_emissive) built by the oracle's restatement."""
    L = lib()
    h = L.orc_scene_build(int(scene_id), float(light_intensity))
    if not h:
        raise ValueError(f"unknown scene {scene_id}")
    try:
        n, d, ne = L.orc_scene_n_prims(h), L.orc_scene_depth(h), L.orc_scene_n_emissive(h)
        prims = np.zeros((n, 64), np.float32)
        nodes = np.zeros((2 ** (d + 1) - 1, 6), np.float32)
        leaves = np.zeros(2 ** d, np.int32)
        L.orc_scene_export(h, P(prims), P(nodes), P(leaves, _ip))
    finally:
        L.orc_scene_free(h)
    return prims, nodes, leaves, d, ne


def custom_scene(ops, light_intensity: float = 1.2):
    """Build a scene from [(type 1..5, trf16 column-major, material7)] with the oracle's own
    producer (scene.h add_* + finalize): (prims, nodes, leaves, depth, nb_emissive)."""
    L = lib()
    h = L.orc_scene_new(ctypes.c_float(light_intensity))
    try:
        for t, trf, mat in ops:
            a = np.ascontiguousarray(trf, np.float32).reshape(16)
            m = np.ascontiguousarray(mat, np.float32).reshape(7)
            if L.orc_scene_add(h, int(t), P(a), P(m)) < 0:
                raise ValueError(f"bad primitive type {t}")
        L.orc_scene_finalize(h)
        n, d = L.orc_scene_n_prims(h), L.orc_scene_depth(h)
        prims = np.zeros((n, 64), np.float32)
        nodes = np.zeros(((2 << d) - 1) * 6, np.float32)
        leaves = np.zeros(1 << d, np.int32)
        L.orc_scene_export(h, P(prims), P(nodes), P(leaves, _ip))
        return prims, nodes, leaves, d, L.orc_scene_n_emissive(h)
    finally:
        L.orc_scene_free(h)


def camera(W: int, H: int) -> Tuple[np.ndarray, np.ndarray]:
    ipv = np.zeros(16, np.float32)
    iv = np.zeros(16, np.float32)
    lib().orc_camera(int(W), int(H), P(ipv), P(iv))
    return ipv, iv


class MeshView:
    """Holds flat mesh buffers (a Scene.mesh_buffers()-style dict) for orc_render/orc_trace."""

    def __init__(self, mb, flat_face=False):
        self.arrays = {k: np.ascontiguousarray(mb[k], np.int32 if k in ("info", "leaves", "tris") else np.float32)
                       for k in ("info", "nodes", "leaves", "tris", "verts", "normals")}
        a = self.arrays
        self.h = lib().orc_mesh_view(P(a["info"], _ip), P(a["nodes"]), P(a["leaves"], _ip), P(a["tris"], _ip),
                                     P(a["verts"]), P(a["normals"]), a["info"].shape[0], int(bool(flat_face)))

    def __del__(self):
        if getattr(self, "h", None) and _L is not None:
            _L.orc_mesh_view_free(self.h)
            self.h = None


def mesh_bvh(verts, tris):
    """Independent mesh BVH (SceneMesh::prim_bb + BVH_KDtree): (depth, nodes, leaves)."""
    v = np.ascontiguousarray(verts, np.float32).reshape(-1, 3)
    t = np.ascontiguousarray(tris, np.int32).reshape(-1, 3)
    d = int(np.ceil(np.log2(np.float32(t.shape[0])))) if t.shape[0] > 1 else 0
    nodes = np.zeros((2 ** (d + 1) - 1, 6), np.float32)
    leaves = np.zeros(2 ** d, np.int32)
    depth = lib().orc_mesh_bvh(P(v), P(t, _ip), t.shape[0], P(nodes), P(leaves, _ip))
    assert depth == d, (depth, d)
    return depth, nodes, leaves


def render(prims, nodes, leaves, depth, invPV, invV, W, H, first_pass=1, n_passes=1, date=0.0,
           bounces=3, ior=1.0, variant=0, row_step=1, row_offset=0, n_threads=0, accum=None, trav_px=None,
           meshes=None):
    """Accumulate passes into accum (H×W×3 f32, row 0 = bottom); returns (accum, events[8]).
    trav_px: optional H×W uint32 array receiving each pixel's traversal count (analysis)."""
    prims = np.ascontiguousarray(prims, np.float32)
    nodes = np.ascontiguousarray(nodes, np.float32)
    leaves = np.ascontiguousarray(leaves, np.int32)
    invPV = np.ascontiguousarray(invPV, np.float32)
    invV = np.ascontiguousarray(invV, np.float32)
    if accum is None:
        accum = np.zeros((H, W, 3), np.float32)
    ev = np.zeros(len(EV_NAMES), np.uint64)
    r = lib().orc_render(P(prims), prims.size // 64, P(nodes), P(leaves, _ip), int(depth), P(invPV), P(invV),
                         int(W), int(H), int(first_pass), int(n_passes), float(date), int(bounces), float(ior),
                         int(variant), int(row_step), int(row_offset), int(n_threads), P(accum), P(ev, _u64p),
                         P(trav_px, _up) if trav_px is not None else None, meshes.h if meshes is not None else None)
    if r != 0:
        raise RuntimeError(f"orc_render failed ({r})")
    return accum, ev


def render_pixels(prims, nodes, leaves, depth, invPV, invV, W, H, xy, first_pass=1, n_passes=1, date=0.0,
                  bounces=3, ior=1.0, variant=0, per_pass=False, n_threads=0):
    """Sums of passes [first_pass, first_pass+n_passes) for an explicit pixel list xy (n × 2 of
    (x, y), row 0 = bottom); returns n × 3 f32.  per_pass=True blends pass by pass in the
    reference's order (montecarlo.cpp:450-466); False follows the chunked accumulation contract
    (bit-equal to render() on the same pixels)."""
    prims = np.ascontiguousarray(prims, np.float32)
    nodes = np.ascontiguousarray(nodes, np.float32)
    leaves = np.ascontiguousarray(leaves, np.int32)
    invPV = np.ascontiguousarray(invPV, np.float32)
    invV = np.ascontiguousarray(invV, np.float32)
    xy = np.ascontiguousarray(np.asarray(xy).reshape(-1, 2), np.int32)
    out = np.zeros((xy.shape[0], 3), np.float32)
    r = lib().orc_render_pixels(P(prims), prims.size // 64, P(nodes), P(leaves, _ip), int(depth), P(invPV), P(invV),
                                int(W), int(H), P(xy, _ip), xy.shape[0], int(first_pass), int(n_passes), float(date),
                                int(bounces), float(ior), int(variant), int(bool(per_pass)), int(n_threads), P(out))
    if r != 0:
        raise RuntimeError(f"orc_render_pixels failed ({r})")
    return out


def xxhash32(x: int, y: int, z: int) -> int:
    return int(lib().orc_xxhash32(x, y, z))


def srand(tcx: float, tcy: float, np_: int, date: float = 0.0) -> np.ndarray:
    s = np.zeros(3, np.uint32)
    lib().orc_srand(float(tcx), float(tcy), int(np_), float(date), P(s, _up))
    return s


def random_floats(seed3, n: int) -> np.ndarray:
    s = np.ascontiguousarray(seed3, np.uint32)
    out = np.zeros(n, np.float32)
    lib().orc_random_floats(P(s, _up), int(n), P(out))
    return out


def sincos(x: float) -> Tuple[float, float]:
    s, c = ctypes.c_float(), ctypes.c_float()
    lib().orc_sincos(float(x), ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def random_ray(seed3, D, roughness: float):
    s = np.ascontiguousarray(seed3, np.uint32)
    d = np.ascontiguousarray(D, np.float32)
    out = np.zeros(3, np.float32)
    so = np.zeros(3, np.uint32)
    lib().orc_random_ray(P(s, _up), P(d), float(roughness), P(out), P(so, _up))
    return out, so


def intersect_prim(rec64, O, D):
    rec = np.ascontiguousarray(rec64, np.float32)
    o = np.ascontiguousarray(O, np.float32)
    d = np.ascontiguousarray(D, np.float32)
    dist = ctypes.c_float()
    dr = ctypes.c_int()
    pl = np.zeros(3, np.float32)
    pg = np.zeros(3, np.float32)
    shape = lib().orc_intersect_prim(P(rec), P(o), P(d), ctypes.byref(dist), ctypes.byref(dr), P(pl), P(pg))
    return shape, dist.value, dr.value, pl, pg


def trace(prims, nodes, leaves, depth, origins, dirs, any_hit=False, prim=-1, meshes=None):
    """(ints n×3 [shape, prim, dir], floats n×21 [dist, pl, pg, N, P, colour, material])."""
    prims = np.ascontiguousarray(prims, np.float32)
    nodes = np.ascontiguousarray(nodes, np.float32)
    leaves = np.ascontiguousarray(leaves, np.int32)
    o = np.ascontiguousarray(np.asarray(origins, np.float32).reshape(-1, 3))
    d = np.ascontiguousarray(np.asarray(dirs, np.float32).reshape(-1, 3))
    n = o.shape[0]
    oi = np.zeros((n, 3), np.int32)
    of = np.zeros((n, 21), np.float32)
    r = lib().orc_trace(P(prims), prims.size // 64, P(nodes), P(leaves, _ip), int(depth), P(o), P(d), n,
                        int(bool(any_hit)), int(prim), P(oi, _ip), P(of), meshes.h if meshes is not None else None)
    if r != 0:
        raise RuntimeError("orc_trace failed")
    return oi, of


def sample_hemisphere(normal, fseed, n, roughness=1.0, nb_used=3):
    out = np.zeros((int(n), 3), np.float32)
    lib().orc_sample_hemisphere(P(np.ascontiguousarray(normal, np.float32)), P(np.ascontiguousarray(fseed, np.float32)),
                                float(roughness), int(nb_used), int(n), P(out))
    return out


def corner_rays(invPV, invV) -> np.ndarray:
    out = np.zeros(15, np.float32)
    lib().orc_corner_rays(P(np.ascontiguousarray(invPV, np.float32)), P(np.ascontiguousarray(invV, np.float32)), P(out))
    return out
