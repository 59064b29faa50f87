"""mcpt — host-side mirror of the reference's render-path API over the libmcpt C ABI.

The product is ``libmcpt.so`` (HIP kernels for gfx950 + C ABI + C++ scene producer,
``../csrc``).  This module is a thin ctypes binding that mirrors the reference's
host interface for the hot path so a user of ``MontecarloGPU/montecarlo.cpp`` finds
the same objects:

* :class:`Scene`     — ``ScenePrimitives`` + ``BVH_GPU_Scene`` (add_*/finalize/depth/
  nb_prim/nb_emissives; bvh_gpu/gpu_bvh_scene.h:35-121) and the 8 reference scenes
  (montecarlo.cpp:629-795);
* :class:`Renderer`  — the GL program + RGB32F accumulation FBO of ``RTViewer``
  (montecarlo.cpp:384-386, 408-477): upload, passes, read-back, average;
* :func:`camera_canonical` — the default camera (camera.cpp:53-95, montecarlo.cpp:405).

There is no CPU fallback: if ``libmcpt.so`` is missing or the GPU is absent, the
calls raise :class:`MCPTError`.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "MCPTError", "lib", "lib_path", "Scene", "Renderer", "camera_canonical",
    "MONTECARLO", "MAT", "MAT_TR", "EVENT_NAMES", "SCENE_KEYS",
    "TRAVERSAL_AUTO", "TRAVERSAL_LANE", "TRAVERSAL_WAVE", "TRAVERSAL_STREAM",
    "Transfo", "average", "write_pfm", "write_png", "material", "light", "Hit", "HIT_DTYPE",
]

MONTECARLO, MAT, MAT_TR = 0, 1, 2
TRAVERSAL_AUTO, TRAVERSAL_LANE, TRAVERSAL_WAVE, TRAVERSAL_STREAM = 0, 1, 2, 3
# launches of one shape AUTO spends on its timing trials before it settles (up to five candidate
# schedules, each timed twice: mcpt_capi.hip kTuneRounds; a trial's time is read when the call
# after the next one starts, so the decision comes two calls after the last trial); callers that
# measure run these first
AUTO_TRIALS = 12
EVENT_NAMES = ("node", "leaf", "prim", "cand", "geom", "colmat", "sample", "trav", "mesh", "tri", "mgeom")
# key bindings of montecarlo.cpp:251-290: scene id -> key
SCENE_KEYS = {1: "Q", 2: "W", 3: "E", 4: "R", 5: "T", 6: "Y", 7: "U", 8: "I"}

_HERE = os.path.dirname(os.path.abspath(__file__))


DEBUG_SLOTS = 64   # MCPT_DEBUG_SLOTS


class MCPTError(RuntimeError):
    pass


class Hit(ctypes.Structure):
    """mcpt_hit (include/mcpt.h): one ray-query result."""
    _fields_ = [("shape", ctypes.c_int), ("prim", ctypes.c_int), ("dir", ctypes.c_int), ("dist", ctypes.c_float),
                ("pl", ctypes.c_float * 3), ("pg", ctypes.c_float * 3), ("N", ctypes.c_float * 3),
                ("P", ctypes.c_float * 3), ("color", ctypes.c_float * 4), ("material", ctypes.c_float * 4)]


HIT_DTYPE = np.dtype([("shape", "<i4"), ("prim", "<i4"), ("dir", "<i4"), ("dist", "<f4"), ("pl", "<f4", 3),
                      ("pg", "<f4", 3), ("N", "<f4", 3), ("P", "<f4", 3), ("color", "<f4", 4),
                      ("material", "<f4", 4)])


def lib_path() -> str:
    return os.environ.get("MCPT_LIB", os.path.join(_HERE, "libmcpt.so"))


_lib: Optional[ctypes.CDLL] = None
_c_float_p = ctypes.POINTER(ctypes.c_float)
_c_int_p = ctypes.POINTER(ctypes.c_int)
_c_u64_p = ctypes.POINTER(ctypes.c_ulonglong)
_vp = ctypes.c_void_p


def _declare(L: ctypes.CDLL) -> None:
    i, f, fp, ip = ctypes.c_int, ctypes.c_float, _c_float_p, _c_int_p
    sig = {
        "mcpt_error_string": (ctypes.c_char_p, [i]),
        "mcpt_version": (i, []),
        "mcpt_build_flags": (i, []),
        "mcpt_create": (i, [i, ctypes.POINTER(_vp)]),
        "mcpt_destroy": (i, [_vp]),
        "mcpt_upload_scene": (i, [_vp, fp, i, fp, ip, i, i]),
        "mcpt_set_target": (i, [_vp, i, i, i, i, i]),
        "mcpt_local_rows": (i, [_vp, ip]),
        "mcpt_set_target_rows": (i, [_vp, i, i, ip, i]),
        "mcpt_balanced_rows": (i, [i, i, i, i, ip, ip]),
        "mcpt_local_row_ids": (i, [_vp, ip]),
        "mcpt_render": (i, [_vp, fp, fp, i, i, f, i, f, i]),
        "mcpt_render_counted": (i, [_vp, fp, fp, i, i, f, i, f, i, _c_u64_p]),
        "mcpt_event_bytes": (i, [i]),
        "mcpt_debug_counters": (i, [_vp, _c_u64_p, i, i]),
        "mcpt_read_accum": (i, [_vp, fp, ip]),
        "mcpt_clear_accum": (i, [_vp]),
        "mcpt_accum_device_ptr": (i, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_size_t)]),
        "mcpt_copy_accum_device": (i, [_vp, _vp, ctypes.c_size_t]),
        "mcpt_gather_rows": (i, [_vp, ctypes.POINTER(_vp), i]),
        "mcpt_set_traversal": (i, [_vp, i]),
        "mcpt_trace": (i, [_vp, fp, fp, i, i, i, _vp]),
        "mcpt_sample_hemisphere": (i, [_vp, fp, fp, f, i, i, fp]),
        "mcpt_get_traversal": (i, [_vp, ip]),
        "mcpt_get_schedule": (i, [_vp, ip, ip, ip]),
        "mcpt_set_walk_exit": (i, [_vp, i]),
        "mcpt_get_walk_exit": (i, [_vp, ip]),
        "mcpt_set_leaf_batch": (i, [_vp, i]),
        "mcpt_get_leaf_batch": (i, [_vp, ip]),
        "mcpt_set_partial_budget": (i, [_vp, ctypes.c_size_t]),
        "mcpt_set_render_lanes": (i, [_vp, i]),
        "mcpt_set_stream_pool": (i, [_vp, i, i]),
        "mcpt_stream_iterations": (i, [_vp, ctypes.POINTER(ctypes.c_longlong)]),
        "mcpt_last_launch_count": (i, [_vp, ip]),
        "mcpt_last_pass_split": (i, [_vp, ip]),
        "mcpt_set_stream": (i, [_vp, _vp]),
        "mcpt_synchronize": (i, [_vp]),
        "mcpt_last_render_ms": (i, [_vp, fp]),
        "mcpt_last_kernel_ms": (i, [_vp, fp, fp]),
        "mcpt_kernel_ms_back": (i, [_vp, ctypes.c_int, fp, fp]),
        "mcpt_kernel_span_ms_back": (i, [_vp, ctypes.c_int, fp]),
        "mcpt_scene_create": (i, [ctypes.POINTER(_vp)]),
        "mcpt_scene_destroy": (i, [_vp]),
        "mcpt_scene_clear": (i, [_vp]),
        "mcpt_scene_add_sphere": (i, [_vp, fp, fp]),
        "mcpt_scene_add_cube": (i, [_vp, fp, fp]),
        "mcpt_scene_add_cylinder": (i, [_vp, fp, fp]),
        "mcpt_scene_add_cone": (i, [_vp, fp, fp]),
        "mcpt_scene_add_oriented_quad": (i, [_vp, fp, fp]),
        "mcpt_scene_finalize": (i, [_vp]),
        "mcpt_scene_add_mesh": (i, [_vp, fp, fp, i, ctypes.POINTER(ctypes.c_uint), i, fp, ip]),
        "mcpt_scene_place_mesh": (i, [_vp, i, fp, fp]),
        "mcpt_scene_mesh_sizes": (i, [_vp, ip, ip, ip, ip, ip]),
        "mcpt_scene_get_mesh_buffers": (i, [_vp, ip, fp, ip, ip, fp, fp]),
        "mcpt_upload_meshes": (i, [_vp, i, ip, i, fp, i, ip, i, ip, i, fp, fp]),
        "mcpt_set_flat_face": (i, [_vp, i]),
        "mcpt_scene_nb_prim": (i, [_vp, ip]),
        "mcpt_scene_depth": (i, [_vp, ip]),
        "mcpt_scene_nb_emissives": (i, [_vp, ip]),
        "mcpt_scene_get_buffers": (i, [_vp, fp, fp, ip]),
        "mcpt_scene_set_material": (i, [_vp, i, fp]),
        "mcpt_scene_build_reference": (i, [_vp, i, f]),
        "mcpt_camera_canonical": (i, [i, i, fp, fp]),
        "mcpt_transfo_translate": (i, [f, f, f, fp]),
        "mcpt_transfo_scale": (i, [f, f, f, fp]),
        "mcpt_transfo_rotate": (i, [i, f, fp]),
        "mcpt_mat4_mul": (i, [fp, fp, fp]),
        "mcpt_average": (i, [fp, ctypes.c_longlong, i, fp]),
        "mcpt_write_pfm": (i, [ctypes.c_char_p, fp, i, i]),
        "mcpt_write_png": (i, [ctypes.c_char_p, fp, i, i]),
        "mcpt_write_accum": (i, [_vp, fp, i]),
        "mcpt_checkpoint_write": (i, [ctypes.c_char_p, fp, i, i, i, i, ctypes.c_char_p]),
        "mcpt_checkpoint_save": (i, [_vp, ctypes.c_char_p, i, ctypes.c_char_p]),
        "mcpt_checkpoint_load": (i, [_vp, ctypes.c_char_p, ctypes.c_char_p, ip]),
        "mcpt_checkpoint_read": (i, [ctypes.c_char_p, fp, ctypes.c_longlong, ip, ip, ip, ip, ctypes.c_char_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args


def lib() -> ctypes.CDLL:
    """Load libmcpt.so (fails loudly: there is no fallback implementation)."""
    global _lib
    if _lib is None:
        path = lib_path()
        if not os.path.exists(path):
            raise MCPTError(f"libmcpt.so not found at {path}: build it with "
                            "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C "
                            "montecarlo-pathtracing_amd/csrc`")
        L = ctypes.CDLL(path)
        _declare(L)
        _lib = L
    return _lib


BUILD_CHECKED, BUILD_STAMPS, BUILD_LANESTATS, BUILD_BLOCKTIMES, BUILD_DRIVER_MATH = 1, 2, 4, 8, 16


def build_flags() -> int:
    """mcpt_build_flags: which diagnostic build the loaded library is (0: the shipped build)."""
    return int(lib().mcpt_build_flags())


def _check(status: int, what: str) -> None:
    if status != 0:
        msg = lib().mcpt_error_string(status).decode()
        raise MCPTError(f"{what} failed ({status}): {msg}")


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_c_float_p)


def _ip(a: np.ndarray):
    return a.ctypes.data_as(_c_int_p)


def _f32(a, n: int) -> np.ndarray:
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1))
    if arr.size != n:
        raise ValueError(f"expected {n} floats, got {arr.size}")
    return arr


def material(rgba: Sequence[float], shininess: float = 0.0, roughness: float = 0.0,
             emissivity: float = 0.0) -> np.ndarray:
    """Material (bvh_gpu/scene.h:30-49) packed as the 7 floats the C ABI takes."""
    return np.array(list(rgba) + [shininess, roughness, emissivity], dtype=np.float32)


def light(rgba: Sequence[float], emissivity: float) -> np.ndarray:
    """Material::light (scene.h:48)."""
    return material(rgba, 0.0, 0.0, emissivity)


class Scene:
    """ScenePrimitives + BVH_GPU_Scene (host side, C++ in libmcpt)."""

    def __init__(self) -> None:
        h = _vp()
        _check(lib().mcpt_scene_create(ctypes.byref(h)), "mcpt_scene_create")
        self._h = h

    def __del__(self) -> None:
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.mcpt_scene_destroy(h)
            self._h = None

    @classmethod
    def reference(cls, scene_id: int, light_intensity: float = 1.2) -> "Scene":
        """Build one of the 8 scenes of montecarlo.cpp (keys Q..I → 1..8), finalized."""
        s = cls()
        _check(lib().mcpt_scene_build_reference(s._h, int(scene_id), float(light_intensity)),
               f"mcpt_scene_build_reference({scene_id})")
        return s

    def clear(self) -> None:
        _check(lib().mcpt_scene_clear(self._h), "mcpt_scene_clear")

    def _add(self, fn: str, trf, mat) -> None:
        t = _f32(trf, 16)
        m = _f32(mat, 7)
        _check(getattr(lib(), fn)(self._h, _fp(t), _fp(m)), fn)

    # transforms are 4x4 column-major (GL / Eigen storage); a (4,4) numpy array in
    # row-major math convention is accepted and transposed to column-major storage.
    @staticmethod
    def _colmajor(trf) -> np.ndarray:
        a = np.asarray(trf, dtype=np.float32)
        return a.T.reshape(-1) if a.shape == (4, 4) else a.reshape(-1)

    def add_sphere(self, trf, mat) -> None:
        self._add("mcpt_scene_add_sphere", self._colmajor(trf), mat)

    def add_cube(self, trf, mat) -> None:
        self._add("mcpt_scene_add_cube", self._colmajor(trf), mat)

    def add_cylinder(self, trf, mat) -> None:
        self._add("mcpt_scene_add_cylinder", self._colmajor(trf), mat)

    def add_cone(self, trf, mat) -> None:
        self._add("mcpt_scene_add_cone", self._colmajor(trf), mat)

    def add_oriented_quad(self, trf, mat) -> None:
        self._add("mcpt_scene_add_oriented_quad", self._colmajor(trf), mat)

    add_orientedQuad = add_oriented_quad   # reference spelling (gpu_bvh_scene.h:103)

    def add_mesh(self, vertices, normals, tri_indices, bb=None) -> int:
        """BVH_GPU_Scene::add_mesh: store a mesh (positions, normals, triangle vertex indices)
        and build its BVH; bb = (min.xyz, max.xyz) of Mesh::BB(), default the vertices' box.
        Returns the mesh id for place_mesh."""
        v = np.ascontiguousarray(np.asarray(vertices, np.float32).reshape(-1, 3))
        n = np.ascontiguousarray(np.asarray(normals, np.float32).reshape(-1, 3))
        t = np.ascontiguousarray(np.asarray(tri_indices, np.uint32).reshape(-1, 3))
        if n.shape != v.shape:
            raise ValueError("one normal per vertex")
        b = None if bb is None else _f32(bb, 6)
        mid = ctypes.c_int()
        _check(lib().mcpt_scene_add_mesh(self._h, _fp(v), _fp(n), v.shape[0],
                                         t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint)), t.shape[0],
                                         _fp(b) if b is not None else None, ctypes.byref(mid)), "mcpt_scene_add_mesh")
        return mid.value

    def place_mesh(self, mesh_id: int, trf, mat) -> None:
        """BVH_GPU_Scene::place_mesh: an instance of mesh `mesh_id` (a CODE_MESH primitive)."""
        t = _f32(self._colmajor(trf), 16)
        m = _f32(mat, 7)
        _check(lib().mcpt_scene_place_mesh(self._h, int(mesh_id), _fp(t), _fp(m)), "mcpt_scene_place_mesh")

    def mesh_buffers(self):
        """dict of the flat mesh buffers (mcpt_scene_get_mesh_buffers layouts), or None."""
        sz = [ctypes.c_int() for _ in range(5)]
        _check(lib().mcpt_scene_mesh_sizes(self._h, *[ctypes.byref(x) for x in sz]), "mcpt_scene_mesh_sizes")
        nm, nn, nl, nt, nv = (x.value for x in sz)
        if nm == 0:
            return None
        b = {"info": np.zeros((nm, 4), np.int32), "nodes": np.zeros((nn, 6), np.float32),
             "leaves": np.zeros(nl, np.int32), "tris": np.zeros((nt, 3), np.int32),
             "verts": np.zeros((nv, 3), np.float32), "normals": np.zeros((nv, 3), np.float32)}
        _check(lib().mcpt_scene_get_mesh_buffers(self._h, _ip(b["info"]), _fp(b["nodes"]), _ip(b["leaves"]),
                                                 _ip(b["tris"]), _fp(b["verts"]), _fp(b["normals"])),
               "mcpt_scene_get_mesh_buffers")
        return b

    def finalize(self) -> None:
        _check(lib().mcpt_scene_finalize(self._h), "mcpt_scene_finalize")

    def nb_prim(self) -> int:
        n = ctypes.c_int()
        _check(lib().mcpt_scene_nb_prim(self._h, ctypes.byref(n)), "mcpt_scene_nb_prim")
        return n.value

    def depth(self, i: int = 0) -> int:
        d = ctypes.c_int()
        _check(lib().mcpt_scene_depth(self._h, ctypes.byref(d)), "mcpt_scene_depth")
        return d.value

    def nb_emissives(self) -> int:
        n = ctypes.c_int()
        _check(lib().mcpt_scene_nb_emissives(self._h, ctypes.byref(n)), "mcpt_scene_nb_emissives")
        return n.value

    def buffers(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(prims n×64 f32, nodes (2^(d+1)-1)×6 f32, leaves 2^d i32) — texture layouts."""
        n, d = self.nb_prim(), self.depth()
        prims = np.zeros((n, 64), np.float32)
        nodes = np.zeros((2 ** (d + 1) - 1, 6), np.float32)
        leaves = np.zeros(2 ** d, np.int32)
        _check(lib().mcpt_scene_get_buffers(self._h, _fp(prims), _fp(nodes), _ip(leaves)),
               "mcpt_scene_get_buffers")
        return prims, nodes, leaves

    def set_material(self, prim: int, mat) -> None:
        m = _f32(mat, 7)
        _check(lib().mcpt_scene_set_material(self._h, int(prim), _fp(m)), "mcpt_scene_set_material")


def camera_canonical(W: int, H: int) -> Tuple[np.ndarray, np.ndarray]:
    """(invPV, invV) of the default camera at aspect W/H, 16 f32 column-major each."""
    ipv = np.zeros(16, np.float32)
    iv = np.zeros(16, np.float32)
    _check(lib().mcpt_camera_canonical(int(W), int(H), _fp(ipv), _fp(iv)), "mcpt_camera_canonical")
    return ipv, iv


# ---- Transfo (easycppogl/gl_eigen.cpp:29-105) and GLMat4 product, computed by libmcpt
def _m16(fn, *args) -> np.ndarray:
    out = np.zeros(16, np.float32)
    _check(getattr(lib(), fn)(*args, _fp(out)), fn)
    return out


class Transfo:
    """Reference Transfo: 4x4 column-major float matrices (16 floats), angles in degrees."""

    @staticmethod
    def translate(x, y, z) -> np.ndarray:
        return _m16("mcpt_transfo_translate", float(x), float(y), float(z))

    @staticmethod
    def scale(sx, sy=None, sz=None) -> np.ndarray:
        sy = sx if sy is None else sy
        sz = sx if sz is None else sz
        return _m16("mcpt_transfo_scale", float(sx), float(sy), float(sz))

    @staticmethod
    def rotateX(deg) -> np.ndarray:
        return _m16("mcpt_transfo_rotate", 0, float(deg))

    @staticmethod
    def rotateY(deg) -> np.ndarray:
        return _m16("mcpt_transfo_rotate", 1, float(deg))

    @staticmethod
    def rotateZ(deg) -> np.ndarray:
        return _m16("mcpt_transfo_rotate", 2, float(deg))

    @staticmethod
    def mul(*ms) -> np.ndarray:
        """Product a * b * ... in the reference's float arithmetic (left to right)."""
        acc = _f32(ms[0], 16)
        for m in ms[1:]:
            b = _f32(m, 16)
            out = np.zeros(16, np.float32)
            _check(lib().mcpt_mat4_mul(_fp(acc), _fp(b), _fp(out)), "mcpt_mat4_mul")
            acc = out
        return acc


# ---- output step
def average(accum: np.ndarray, pass_count: int) -> np.ndarray:
    """fs_frag: accum / nb (montecarlo.cpp:59-70), binary32 per channel."""
    a = np.ascontiguousarray(accum, np.float32)
    out = np.empty_like(a)
    _check(lib().mcpt_average(_fp(a), a.size, int(pass_count), _fp(out)), "mcpt_average")
    return out


def write_pfm(path: str, rgb: np.ndarray) -> None:
    a = np.ascontiguousarray(rgb, np.float32)
    _check(lib().mcpt_write_pfm(str(path).encode(), _fp(a), a.shape[1], a.shape[0]), "mcpt_write_pfm")


def write_png(path: str, rgb: np.ndarray) -> None:
    """8-bit framebuffer view: clamp [0,1], round(255·c), no gamma (GL unorm conversion)."""
    a = np.ascontiguousarray(rgb, np.float32)
    _check(lib().mcpt_write_png(str(path).encode(), _fp(a), a.shape[1], a.shape[0]), "mcpt_write_png")


# ---- checkpoint / resume of a progressive render (mcpt.h: mcpt_checkpoint_write / _read)
CHECKPOINT_TAG_MAX = 1024


def checkpoint_write(path: str, accum: np.ndarray, pass_count: int, next_pass: int, tag: str = "") -> None:
    """accum: rows × W × 3 f32 sums holding `pass_count` passes; `next_pass` = the first pass
    of the render call that continues; `tag` = the render parameters the reader compares."""
    a = np.ascontiguousarray(accum, np.float32)
    if a.ndim != 3 or a.shape[2] != 3:
        raise MCPTError("checkpoint_write: accum must be rows x W x 3")
    _check(lib().mcpt_checkpoint_write(str(path).encode(), _fp(a), a.shape[1], a.shape[0], int(pass_count),
                                       int(next_pass), tag.encode()), "mcpt_checkpoint_write")


def checkpoint_read(path: str) -> Tuple[np.ndarray, int, int, str]:
    """(accum rows × W × 3, pass_count, next_pass, tag) of a checkpoint file."""
    w, rows, pc, nxt = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    tag = ctypes.create_string_buffer(CHECKPOINT_TAG_MAX)
    _check(lib().mcpt_checkpoint_read(str(path).encode(), None, 0, ctypes.byref(w), ctypes.byref(rows), None, None,
                                      None), "mcpt_checkpoint_read")
    out = np.empty((rows.value, w.value, 3), np.float32)
    # the capacity bounds the read if the file was replaced in between; the shape is re-read
    _check(lib().mcpt_checkpoint_read(str(path).encode(), _fp(out), out.size, ctypes.byref(w), ctypes.byref(rows),
                                      ctypes.byref(pc), ctypes.byref(nxt), tag), "mcpt_checkpoint_read")
    if (rows.value, w.value, 3) != out.shape:
        raise MCPTError("checkpoint_read: the file changed while it was read")
    return out, pc.value, nxt.value, tag.value.decode()


class Renderer:
    """Device context: scene on the GPU, row-band framebuffer, pass accumulation."""

    def __init__(self, device: int = 0) -> None:
        h = _vp()
        _check(lib().mcpt_create(int(device), ctypes.byref(h)), "mcpt_create")
        self._h = h
        self.W = self.H = 0
        self.band_rows, self.world, self.rank = 1, 1, 0
        self.n_local_rows = 0

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().mcpt_destroy(self._h)
            self._h = None

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:
            pass

    def upload_scene(self, scene: Optional[Scene] = None, prims=None, nodes=None, leaves=None,
                     depth: Optional[int] = None, nb_emissives: int = 0) -> None:
        if scene is not None:
            prims, nodes, leaves = scene.buffers()
            depth = scene.depth()
            nb_emissives = scene.nb_emissives()
        prims = np.ascontiguousarray(prims, dtype=np.float32)
        nodes = np.ascontiguousarray(nodes, dtype=np.float32)
        leaves = np.ascontiguousarray(leaves, dtype=np.int32)
        n = prims.size // 64
        _check(lib().mcpt_upload_scene(self._h, _fp(prims), int(n), _fp(nodes), _ip(leaves),
                                       int(depth), int(nb_emissives)), "mcpt_upload_scene")
        if scene is not None:
            mb = scene.mesh_buffers()
            if mb is not None:
                self.upload_meshes(mb)

    def upload_meshes(self, mb) -> None:
        """mcpt_upload_meshes from a Scene.mesh_buffers() dict (None/empty: no meshes)."""
        if not mb:
            _check(lib().mcpt_upload_meshes(self._h, 0, None, 0, None, 0, None, 0, None, 0, None, None),
                   "mcpt_upload_meshes")
            return
        info = np.ascontiguousarray(mb["info"], np.int32)
        nodes = np.ascontiguousarray(mb["nodes"], np.float32)
        leaves = np.ascontiguousarray(mb["leaves"], np.int32)
        tris = np.ascontiguousarray(mb["tris"], np.int32)
        verts = np.ascontiguousarray(mb["verts"], np.float32)
        norms = np.ascontiguousarray(mb["normals"], np.float32)
        _check(lib().mcpt_upload_meshes(self._h, info.shape[0], _ip(info), nodes.shape[0], _fp(nodes), leaves.size,
                                        _ip(leaves), tris.shape[0], _ip(tris), verts.shape[0], _fp(verts),
                                        _fp(norms)), "mcpt_upload_meshes")

    def set_flat_face(self, flat: bool) -> None:
        _check(lib().mcpt_set_flat_face(self._h, int(bool(flat))), "mcpt_set_flat_face")

    def set_target(self, W: int, H: int, band_rows: int = 8, world: int = 1, rank: int = 0) -> None:
        _check(lib().mcpt_set_target(self._h, int(W), int(H), int(band_rows), int(world), int(rank)),
               "mcpt_set_target")
        self.W, self.H = int(W), int(H)
        self.band_rows, self.world, self.rank = int(band_rows), int(world), int(rank)
        n = ctypes.c_int()
        _check(lib().mcpt_local_rows(self._h, ctypes.byref(n)), "mcpt_local_rows")
        self.n_local_rows = n.value

    def set_target_rows(self, W: int, H: int, rows) -> None:
        """Explicit shard (mcpt_set_target_rows): local row i renders global row rows[i]."""
        r = np.ascontiguousarray(rows, dtype=np.int32)
        _check(lib().mcpt_set_target_rows(self._h, int(W), int(H), _ip(r), int(r.size)), "mcpt_set_target_rows")
        self.W, self.H = int(W), int(H)
        self.band_rows, self.world, self.rank = 0, 0, 0
        self.n_local_rows = int(r.size)

    def local_row_ids(self) -> np.ndarray:
        out = np.zeros(self.n_local_rows, np.int32)
        if self.n_local_rows:
            _check(lib().mcpt_local_row_ids(self._h, _ip(out)), "mcpt_local_row_ids")
        return out.astype(np.int64)

    def render(self, invPV, invV, first_pass: int, n_passes: int, date: float = 0.0,
               bounces: int = 3, refract_ind: float = 1.0, variant: int = MONTECARLO) -> None:
        a, b = _f32(invPV, 16), _f32(invV, 16)
        _check(lib().mcpt_render(self._h, _fp(a), _fp(b), int(first_pass), int(n_passes), float(date),
                                 int(bounces), float(refract_ind), int(variant)), "mcpt_render")

    def render_counted(self, invPV, invV, first_pass: int, n_passes: int, date: float = 0.0,
                       bounces: int = 3, refract_ind: float = 1.0, variant: int = MONTECARLO) -> np.ndarray:
        a, b = _f32(invPV, 16), _f32(invV, 16)
        ev = np.zeros(len(EVENT_NAMES), np.uint64)
        _check(lib().mcpt_render_counted(self._h, _fp(a), _fp(b), int(first_pass), int(n_passes),
                                         float(date), int(bounces), float(refract_ind), int(variant),
                                         ev.ctypes.data_as(_c_u64_p)), "mcpt_render_counted")
        return ev

    def debug_counters(self, reset: bool = True) -> np.ndarray:
        """The context's MCPT_DEBUG_SLOTS device counter slots (diagnostic builds write there)."""
        out = np.zeros(DEBUG_SLOTS, np.uint64)
        _check(lib().mcpt_debug_counters(self._h, out.ctypes.data_as(_c_u64_p), out.size, int(reset)),
               "mcpt_debug_counters")
        return out

    @staticmethod
    def event_bytes() -> np.ndarray:
        return np.array([lib().mcpt_event_bytes(e) for e in range(len(EVENT_NAMES))], np.int64)

    def read_accum(self) -> Tuple[np.ndarray, int]:
        """(local rows × W × 3 f32 sums, pass count)."""
        out = np.zeros((self.n_local_rows, self.W, 3), np.float32)
        pc = ctypes.c_int()
        _check(lib().mcpt_read_accum(self._h, _fp(out), ctypes.byref(pc)), "mcpt_read_accum")
        return out, pc.value

    def read_image(self) -> np.ndarray:
        """Averaged image (fs_frag: accum / nb, montecarlo.cpp:59-70); single-shard only."""
        acc, n = self.read_accum()
        full = self.n_local_rows == self.H and (self.world != 0 or
                                                np.array_equal(self.local_row_ids(), np.arange(self.H)))
        if not full:
            raise MCPTError("read_image needs the full frame in row order; gather shards with mcpt.dist")
        return acc / max(n, 1)

    def clear_accum(self) -> None:
        _check(lib().mcpt_clear_accum(self._h), "mcpt_clear_accum")

    def write_accum(self, accum: np.ndarray, pass_count: int) -> None:
        """mcpt_write_accum: load local rows × W × 3 sums holding `pass_count` passes."""
        a = np.ascontiguousarray(accum, np.float32)
        if a.shape != (self.n_local_rows, self.W, 3):
            raise MCPTError(f"write_accum: expected {(self.n_local_rows, self.W, 3)}, got {a.shape}")
        _check(lib().mcpt_write_accum(self._h, _fp(a), int(pass_count)), "mcpt_write_accum")

    def save_checkpoint(self, path: str, next_pass: int, tag: str = "") -> None:
        """mcpt_checkpoint_save: this context's accumulator, its pass count, `next_pass`, `tag` and
        the target's identity (H, row ids) to `path`."""
        _check(lib().mcpt_checkpoint_save(self._h, str(path).encode(), int(next_pass), tag.encode()),
               "mcpt_checkpoint_save")

    def load_checkpoint(self, path: str, tag: Optional[str] = None) -> int:
        """mcpt_checkpoint_load: resume from `path` — it must have been saved for this target
        (W, H, row ids) and, if `tag` is given, with that tag; loads the sums and pass count and
        returns the first pass of the next render call."""
        nxt = ctypes.c_int()
        _check(lib().mcpt_checkpoint_load(self._h, str(path).encode(), None if tag is None else tag.encode(),
                                          ctypes.byref(nxt)), "mcpt_checkpoint_load")
        return nxt.value

    def accum_device_ptr(self) -> Tuple[int, int]:
        p = _vp()
        n = ctypes.c_size_t()
        _check(lib().mcpt_accum_device_ptr(self._h, ctypes.byref(p), ctypes.byref(n)), "mcpt_accum_device_ptr")
        return int(p.value or 0), int(n.value)

    def copy_accum_device(self, dst_ptr: int, nbytes: int) -> None:
        """D2D copy of the local accumulator into a device buffer (ordered on our stream)."""
        _check(lib().mcpt_copy_accum_device(self._h, _vp(dst_ptr), ctypes.c_size_t(nbytes)),
               "mcpt_copy_accum_device")

    def gather_rows(self, shards) -> None:
        """This full-frame renderer's accumulator <- the shard renderers' rows (mcpt_gather_rows:
        device-to-device peer copies inside one process, ordered after the shards' renders)."""
        hs = (_vp * max(len(shards), 1))(*[s._h for s in shards])
        _check(lib().mcpt_gather_rows(self._h, hs, len(shards)), "mcpt_gather_rows")

    def trace(self, origins, dirs, any_hit: bool = False, prim: int = -1) -> np.ndarray:
        """Ray queries (traverse_all_bvh / just_hit_bvh, or one primitive) + intersection_info.
        Returns a structured array of HIT_DTYPE records (shape -1 = miss)."""
        o = np.ascontiguousarray(np.asarray(origins, np.float32).reshape(-1, 3))
        d = np.ascontiguousarray(np.asarray(dirs, np.float32).reshape(-1, 3))
        if o.shape != d.shape:
            raise ValueError("origins and dirs must have the same shape")
        out = np.zeros(o.shape[0], HIT_DTYPE)
        assert HIT_DTYPE.itemsize == ctypes.sizeof(Hit)
        _check(lib().mcpt_trace(self._h, _fp(o), _fp(d), o.shape[0], int(bool(any_hit)), int(prim),
                                out.ctypes.data_as(_vp)), "mcpt_trace")
        return out

    def sample_hemisphere(self, normal, fseed, n: int, roughness: float = 1.0, nb_used: int = 3) -> np.ndarray:
        """DrawSampling point cloud: n directions random_ray(normalize(normal), roughness)."""
        nrm = _f32(normal, 3)
        sd = _f32(fseed, 3)
        out = np.zeros((int(n), 3), np.float32)
        _check(lib().mcpt_sample_hemisphere(self._h, _fp(nrm), _fp(sd), float(roughness), int(nb_used), int(n),
                                            _fp(out)), "mcpt_sample_hemisphere")
        return out

    def set_traversal(self, mode: int) -> None:
        """BVH traversal strategy: TRAVERSAL_AUTO / _LANE / _WAVE / _STREAM (same results)."""
        _check(lib().mcpt_set_traversal(self._h, int(mode)), "mcpt_set_traversal")

    def set_walk_exit(self, lanes: int) -> None:
        """mcpt_set_walk_exit: suspend per-lane walks at <= lanes walking lanes (-1: default)."""
        _check(lib().mcpt_set_walk_exit(self._h, int(lanes)), "mcpt_set_walk_exit")

    def walk_exit(self) -> int:
        n = ctypes.c_int()
        _check(lib().mcpt_get_walk_exit(self._h, ctypes.byref(n)), "mcpt_get_walk_exit")
        return n.value

    def set_leaf_batch(self, lanes: int) -> None:
        """mcpt_set_leaf_batch: primitive-test block once >= lanes lanes wait on a leaf (-1: default)."""
        _check(lib().mcpt_set_leaf_batch(self._h, int(lanes)), "mcpt_set_leaf_batch")

    def leaf_batch(self) -> int:
        n = ctypes.c_int()
        _check(lib().mcpt_get_leaf_batch(self._h, ctypes.byref(n)), "mcpt_get_leaf_batch")
        return n.value

    def set_stream_pool(self, slots: int = 0, refill: int = -1) -> None:
        """Stream schedule knobs (mcpt_set_stream_pool): path slots (0 = default) and the trace
        kernel's refill threshold (-1 = default).  Same results for every value."""
        _check(lib().mcpt_set_stream_pool(self._h, int(slots), int(refill)), "mcpt_set_stream_pool")

    def stream_iterations(self) -> int:
        """Iterations (trace + shade kernel pairs) of the last stream-schedule launch."""
        n = ctypes.c_longlong()
        _check(lib().mcpt_stream_iterations(self._h, ctypes.byref(n)), "mcpt_stream_iterations")
        return n.value

    def set_partial_budget(self, nbytes: int) -> None:
        """mcpt_set_partial_budget: bound of one launch's segment-sum buffer (calls spanning more
        32-pass chunks are split into launches at chunk boundaries; same bits)."""
        _check(lib().mcpt_set_partial_budget(self._h, int(nbytes)), "mcpt_set_partial_budget")

    def set_render_lanes(self, on: bool) -> None:
        """mcpt_set_render_lanes: consecutive launches on two alternating lanes (overlapping each
        other's tails; the default) or every launch in order on the context's stream."""
        _check(lib().mcpt_set_render_lanes(self._h, int(bool(on))), "mcpt_set_render_lanes")

    def last_launch_count(self) -> int:
        """Sub-launches the last render call was split into."""
        n = ctypes.c_int()
        _check(lib().mcpt_last_launch_count(self._h, ctypes.byref(n)), "mcpt_last_launch_count")
        return n.value

    def last_pass_split(self) -> bool:
        """mcpt_last_pass_split: the last render call ran one segment per pass (small launches;
        same bits)."""
        n = ctypes.c_int()
        _check(lib().mcpt_last_pass_split(self._h, ctypes.byref(n)), "mcpt_last_pass_split")
        return bool(n.value)

    def traversal(self) -> int:
        """The strategy AUTO resolves to for the uploaded scene."""
        m = ctypes.c_int()
        _check(lib().mcpt_get_traversal(self._h, ctypes.byref(m)), "mcpt_get_traversal")
        return m.value

    def schedule(self) -> dict:
        """The schedule of the next launch of the last launch shape (mcpt_get_schedule):
        traversal ("lane"/"wave"/"stream"), pass segments per work item, AUTO settled or not."""
        t, k, s = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib().mcpt_get_schedule(self._h, ctypes.byref(t), ctypes.byref(k), ctypes.byref(s)),
               "mcpt_get_schedule")
        return {"traversal": {1: "lane", 2: "wave", 3: "stream"}.get(t.value, str(t.value)), "seg_per_item": k.value,
                "settled": bool(s.value)}

    def set_stream(self, hip_stream_ptr: int) -> None:
        _check(lib().mcpt_set_stream(self._h, _vp(hip_stream_ptr)), "mcpt_set_stream")

    def synchronize(self) -> None:
        _check(lib().mcpt_synchronize(self._h), "mcpt_synchronize")

    def last_render_ms(self) -> float:
        ms = ctypes.c_float()
        _check(lib().mcpt_last_render_ms(self._h, ctypes.byref(ms)), "mcpt_last_render_ms")
        return ms.value

    def last_kernel_ms(self) -> Tuple[float, float]:
        """(path-tracing kernel ms, chunk-combine kernel ms) of the last render."""
        a, b = ctypes.c_float(), ctypes.c_float()
        _check(lib().mcpt_last_kernel_ms(self._h, ctypes.byref(a), ctypes.byref(b)), "mcpt_last_kernel_ms")
        return a.value, b.value

    # render calls whose kernel times a context keeps (mcpt_kernel_ms_back)
    TIMING_RING = 64

    def kernel_span_ms_back(self, back: int) -> float:
        """mcpt_kernel_span_ms_back: the path-tracing kernel's whole span (own start -> end) of the
        call `back` calls before the last; with render lanes the launches overlap, and
        kernel_ms_back charges each its period instead."""
        a = ctypes.c_float()
        _check(lib().mcpt_kernel_span_ms_back(self._h, int(back), ctypes.byref(a)), "mcpt_kernel_span_ms_back")
        return a.value

    def kernel_ms_back(self, back: int) -> Tuple[float, float]:
        """mcpt_kernel_ms_back: (path-tracing ms, combine ms) of the render call `back` calls
        before the last (0: the last; < TIMING_RING); waits for that call only."""
        a, b = ctypes.c_float(), ctypes.c_float()
        _check(lib().mcpt_kernel_ms_back(self._h, int(back), ctypes.byref(a), ctypes.byref(b)), "mcpt_kernel_ms_back")
        return a.value, b.value
