"""Independent numpy restatement of the reference's HOST producer of the hot path's inputs
(test infrastructure; round 5, verdict r04 item 6): the scene builders, Transfo, the primitive
records, prim_bb, sortEmissiveFirst, the median-split BVH and the canonical camera, written from
the reference's C++ text — not from oracle/oracle.cpp and not from the product's
csrc/mcpt_scene.cpp — so that tests/golden/paths.npz no longer takes its scene buffers and
camera from the oracle.  tests/test_host_producer.py checks all three producers bit for bit.

Reference (citations relative to /root/reference):
  * Transfo::translate / scale / rotateX/Y/Z     easycppogl/gl_eigen.cpp:29-123
  * Transfo::apply                               easycppogl/gl_eigen.h:91-94
  * Material, PrimData, ScenePrimitives::add_*   bvh_gpu/scene.h:30-172
  * add_prim, prim_bb, sortEmissiveFirst, merge  bvh_gpu/scene.cpp:18-100
  * BVH_KDtree::init / split_step / compute      bvh_gpu/bvh.cpp:5-93 (std::nth_element: libstdc++'s
                                                 introselect, restated below)
  * scenes, menger, colours, OPA                 MontecarloGPU/montecarlo.cpp:33-46, 143-180, 629-795
  * camera                                       easycppogl/camera.cpp:28-95, camera.h:62-93,
                                                 montecarlo.cpp:389, 404-405, 439-440

Arithmetic: binary32 everywhere the reference computes in float; Eigen's lazy
float products (the -msse4 build, no FMA) as plain sums in k order; the 4x4 inverse as the
adjugate in binary64 rounded to binary32 (Eigen's SSE float inverse is not reproducible without
Eigen); sin / cos of the rotations from the C library's sinf / cosf (std::sin(float)); the camera
in binary64, cast to binary32 where the reference casts.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

F = np.float32
_libm = ctypes.CDLL("libm.so.6")
for _fn in ("sinf", "cosf"):
    getattr(_libm, _fn).restype = ctypes.c_float
    getattr(_libm, _fn).argtypes = [ctypes.c_float]


def sinf(x):
    return F(_libm.sinf(float(F(x))))


def cosf(x):
    return F(_libm.cosf(float(F(x))))


# ------------------------------------------------------------------------------------------
# GLMat4 (4x4 float, m[r, c]) and Transfo — gl_eigen.cpp:29-123
# ------------------------------------------------------------------------------------------
def ident():
    return np.eye(4, dtype=F)


def translate(x, y, z):
    m = ident()
    m[0, 3], m[1, 3], m[2, 3] = F(x), F(y), F(z)
    return m


def scale(sx, sy=None, sz=None):
    m = ident()
    sy = sx if sy is None else sy
    sz = sx if sz is None else sz
    m[0, 0], m[1, 1], m[2, 2] = F(sx), F(sy), F(sz)
    return m


def _deg(a):
    return F(F(math.pi / 180) * F(a))   # float(M_PI / 180) * a


def rotateX(a):
    al = _deg(a)
    s, c = sinf(al), cosf(al)
    m = ident()
    m[1, 1], m[2, 1], m[1, 2], m[2, 2] = c, s, F(-s), c
    return m


def rotateY(a):
    al = _deg(a)
    s, c = sinf(al), cosf(al)
    m = ident()
    m[0, 0], m[2, 0], m[0, 2], m[2, 2] = c, F(-s), s, c
    return m


def rotateZ(a):
    al = _deg(a)
    s, c = sinf(al), cosf(al)
    m = ident()
    m[0, 0], m[1, 0], m[0, 1], m[1, 1] = c, s, F(-s), c
    return m


def mul(*ms):
    """A * B * ... left to right; each coefficient a plain sum in k order (Eigen's lazy float
    product without FMA)."""
    acc = ms[0]
    for B in ms[1:]:
        R = np.zeros((4, 4), F)
        for i in range(4):
            for j in range(4):
                s = F(acc[i, 0] * B[0, j])
                for k in range(1, 4):
                    s = F(s + F(acc[i, k] * B[k, j]))
                R[i, j] = s
        acc = R
    return acc


def apply4(A, v):
    out = np.zeros(4, F)
    for i in range(4):
        s = F(A[i, 0] * F(v[0]))
        for k in range(1, 4):
            s = F(s + F(A[i, k] * F(v[k])))
        out[i] = s
    return out


def apply(A, p):   # gl_eigen.h:91-94: (tr * (p, 1)).xyz
    return apply4(A, (p[0], p[1], p[2], 1.0))[:3]


def inverse(A):
    """Adjugate (cofactor expansion) in binary64 of the float matrix, / det, rounded to binary32."""
    a = [float(A[k % 4, k // 4]) for k in range(16)]   # column-major a[c*4 + r]
    inv = [0.0] * 16
    inv[0] = a[5] * a[10] * a[15] - a[5] * a[11] * a[14] - a[9] * a[6] * a[15] + a[9] * a[7] * a[14] + a[13] * a[6] * a[11] - a[13] * a[7] * a[10]
    inv[4] = -a[4] * a[10] * a[15] + a[4] * a[11] * a[14] + a[8] * a[6] * a[15] - a[8] * a[7] * a[14] - a[12] * a[6] * a[11] + a[12] * a[7] * a[10]
    inv[8] = a[4] * a[9] * a[15] - a[4] * a[11] * a[13] - a[8] * a[5] * a[15] + a[8] * a[7] * a[13] + a[12] * a[5] * a[11] - a[12] * a[7] * a[9]
    inv[12] = -a[4] * a[9] * a[14] + a[4] * a[10] * a[13] + a[8] * a[5] * a[14] - a[8] * a[6] * a[13] - a[12] * a[5] * a[10] + a[12] * a[6] * a[9]
    inv[1] = -a[1] * a[10] * a[15] + a[1] * a[11] * a[14] + a[9] * a[2] * a[15] - a[9] * a[3] * a[14] - a[13] * a[2] * a[11] + a[13] * a[3] * a[10]
    inv[5] = a[0] * a[10] * a[15] - a[0] * a[11] * a[14] - a[8] * a[2] * a[15] + a[8] * a[3] * a[14] + a[12] * a[2] * a[11] - a[12] * a[3] * a[10]
    inv[9] = -a[0] * a[9] * a[15] + a[0] * a[11] * a[13] + a[8] * a[1] * a[15] - a[8] * a[3] * a[13] - a[12] * a[1] * a[11] + a[12] * a[3] * a[9]
    inv[13] = a[0] * a[9] * a[14] - a[0] * a[10] * a[13] - a[8] * a[1] * a[14] + a[8] * a[2] * a[13] + a[12] * a[1] * a[10] - a[12] * a[2] * a[9]
    inv[2] = a[1] * a[6] * a[15] - a[1] * a[7] * a[14] - a[5] * a[2] * a[15] + a[5] * a[3] * a[14] + a[13] * a[2] * a[7] - a[13] * a[3] * a[6]
    inv[6] = -a[0] * a[6] * a[15] + a[0] * a[7] * a[14] + a[4] * a[2] * a[15] - a[4] * a[3] * a[14] - a[12] * a[2] * a[7] + a[12] * a[3] * a[6]
    inv[10] = a[0] * a[5] * a[15] - a[0] * a[7] * a[13] - a[4] * a[1] * a[15] + a[4] * a[3] * a[13] + a[12] * a[1] * a[7] - a[12] * a[3] * a[5]
    inv[14] = -a[0] * a[5] * a[14] + a[0] * a[6] * a[13] + a[4] * a[1] * a[14] - a[4] * a[2] * a[13] - a[12] * a[1] * a[6] + a[12] * a[2] * a[5]
    inv[3] = -a[1] * a[6] * a[11] + a[1] * a[7] * a[10] + a[5] * a[2] * a[11] - a[5] * a[3] * a[10] - a[9] * a[2] * a[7] + a[9] * a[3] * a[6]
    inv[7] = a[0] * a[6] * a[11] - a[0] * a[7] * a[10] - a[4] * a[2] * a[11] + a[4] * a[3] * a[10] + a[8] * a[2] * a[7] - a[8] * a[3] * a[6]
    inv[11] = -a[0] * a[5] * a[11] + a[0] * a[7] * a[9] + a[4] * a[1] * a[11] - a[4] * a[3] * a[9] - a[8] * a[1] * a[7] + a[8] * a[3] * a[5]
    inv[15] = a[0] * a[5] * a[10] - a[0] * a[6] * a[9] - a[4] * a[1] * a[10] + a[4] * a[2] * a[9] + a[8] * a[1] * a[6] - a[8] * a[2] * a[5]
    det = a[0] * inv[0] + a[1] * inv[4] + a[2] * inv[8] + a[3] * inv[12]
    R = np.zeros((4, 4), F)
    for k in range(16):
        R[k % 4, k // 4] = F(inv[k] / det)
    return R


def colmajor(m):
    return np.ascontiguousarray(m.T).reshape(-1)


# ------------------------------------------------------------------------------------------
# Eigen float vector helpers (no FMA; sums left to right)
# ------------------------------------------------------------------------------------------
def vsub(a, b):
    return np.array([F(a[k] - b[k]) for k in range(3)], F)


def dot(a, b):
    return F(F(F(a[0] * b[0]) + F(a[1] * b[1])) + F(a[2] * b[2]))


def norm(a):
    return F(np.sqrt(dot(a, a)))


def cross(a, b):
    return np.array([F(F(a[1] * b[2]) - F(a[2] * b[1])), F(F(a[2] * b[0]) - F(a[0] * b[2])),
                     F(F(a[0] * b[1]) - F(a[1] * b[0]))], F)


# ------------------------------------------------------------------------------------------
# ScenePrimitives — scene.h:75-172, scene.cpp:18-88
# ------------------------------------------------------------------------------------------
class Material:   # scene.h:30-49
    def __init__(self, color, shin=0.0, rough=0.0, emi=0.0):
        self.color = np.asarray(color, F)
        self.shin, self.rough, self.emi = F(shin), F(rough), F(emi)

    @staticmethod
    def light(color, emi):
        return Material(color, 0.0, 0.0, emi)


class Scene:
    def __init__(self):
        self.recs = []   # PrimData as 64 floats: transfo, inverse, mesh-BB transfo, type, colour, mat_info, padding

    def add_prim(self, prim, trf, mat, area):   # scene.cpp:44-53
        r = np.zeros(64, F)
        r[0:16], r[16:32], r[32:48] = colmajor(trf), colmajor(inverse(trf)), colmajor(trf)
        r[48] = F(prim)
        r[52:56] = mat.color
        r[56], r[57], r[58], r[59] = mat.shin, mat.rough, mat.emi, F(area)
        self.recs.append(r)

    def _uvw(self, trf):
        o = apply(trf, (-1, -1, -1))
        return (vsub(apply(trf, (1, -1, -1)), o), vsub(apply(trf, (-1, 1, -1)), o), vsub(apply(trf, (-1, -1, 1)), o))

    def add_sphere(self, trf, mat):   # scene.h:128-133
        r = norm(np.array([trf[0, 0], trf[1, 0], trf[2, 0]], F))
        self.add_prim(1, trf, mat, F(F(F(2.0 * math.pi) * r) * r))

    def add_cube(self, trf, mat):     # scene.h:135-142
        U, V, W = self._uvw(trf)
        area = F(F(2.0) * F(F(norm(cross(U, V)) + norm(cross(U, W))) + norm(cross(W, V))))
        self.add_prim(2, trf, mat, area)

    def add_cylinder(self, trf, mat):  # scene.h:144-152
        U, V, W = self._uvw(trf)
        area = F(F(F(F(F(dot(U, U) + dot(V, V)) / F(4.0)) * F(np.sqrt(F(2.0)))) * F(math.pi)) * norm(W))
        self.add_prim(3, trf, mat, area)

    def add_cone(self, trf, mat):      # scene.h:154-163 (area TODO in the reference: 0)
        self.add_prim(4, trf, mat, 0.0)

    def add_orientedQuad(self, trf, mat):   # scene.h:166-172
        o = apply(trf, (-1, -1, 0))
        U, V = vsub(apply(trf, (1, -1, 0)), o), vsub(apply(trf, (-1, 1, 0)), o)
        self.add_prim(5, trf, mat, norm(cross(U, V)))

    def sort_emissive_first(self):   # scene.cpp:70-88
        b = self.recs
        nxt = 0
        while nxt < len(b) and b[nxt][58] > 0.0:
            nxt += 1
        for it in range(nxt, len(b)):
            if b[it][58] > 0.0:
                b[nxt], b[it] = b[it], b[nxt]
                nxt += 1
        return nxt

    def prim_bb(self, p):   # scene.cpp:18-42 -> (centre, (min, max))
        rec = self.recs[p]
        t = rec[0:16].reshape(4, 4).T
        lo = np.full(3, np.finfo(F).max, F)
        hi = np.full(3, np.finfo(F).min, F)
        for v in range(8):
            x = F(F(F(v & 1) * F(2.01)) - F(1.005))
            y = F(F(F((v >> 1) & 1) * F(2.01)) - F(1.005))
            z = F(F(F((v >> 2) & 1) * F(2.01)) - F(1.005))
            if rec[48] == F(5.0):
                z = F(z / F(abs(z) * F(1000.0)))
            B = apply4(t, (x, y, z, 1.0))
            for i in range(3):
                if B[i] < lo[i]:
                    lo[i] = B[i]
                if B[i] > hi[i]:
                    hi[i] = B[i]
        return np.array([F(F(lo[i] + hi[i]) / F(2.0)) for i in range(3)], F), (lo, hi)

    def finalize(self):
        """BVH_GPU_Scene::finalize (gpu_bvh_scene.cpp:121-187) on the prims: (prims n x 64,
        nodes (2^(d+1)-1) x 6 (min, max), leaves 2^d, depth, nb_emissive)."""
        nb_emi = self.sort_emissive_first()
        n = len(self.recs)
        cb = [self.prim_bb(i) for i in range(n)]
        centers = [c for c, _ in cb]
        bbs = [np.concatenate(b) for _, b in cb]
        depth, nodes, leaves = kd_tree(centers, bbs)
        return np.stack(self.recs), nodes, leaves, depth, nb_emi


# ------------------------------------------------------------------------------------------
# std::nth_element (libstdc++: introselect, median-of-three pivot, insertion sort below 4,
# heap select past the depth limit), restated on a Python list with comp(a, b) -> bool
# ------------------------------------------------------------------------------------------
def _insertion_sort(v, first, last, comp):
    if first == last:
        return
    for i in range(first + 1, last):
        val = v[i]
        if comp(val, v[first]):
            v[first + 1:i + 1] = v[first:i]
            v[first] = val
        else:
            j = i
            while comp(val, v[j - 1]):
                v[j] = v[j - 1]
                j -= 1
            v[j] = val


def _move_median_to_first(v, result, a, b, c, comp):
    if comp(v[a], v[b]):
        if comp(v[b], v[c]):
            m = b
        elif comp(v[a], v[c]):
            m = c
        else:
            m = a
    elif comp(v[a], v[c]):
        m = a
    elif comp(v[b], v[c]):
        m = c
    else:
        m = b
    v[result], v[m] = v[m], v[result]


def _unguarded_partition(v, first, last, pivot, comp):
    while True:
        while comp(v[first], v[pivot]):
            first += 1
        last -= 1
        while comp(v[pivot], v[last]):
            last -= 1
        if not first < last:
            return first
        v[first], v[last] = v[last], v[first]
        first += 1


def _adjust_heap(v, first, hole, length, value, comp):
    top = hole
    second = hole
    while second < (length - 1) // 2:
        second = 2 * (second + 1)
        if comp(v[first + second], v[first + second - 1]):
            second -= 1
        v[first + hole] = v[first + second]
        hole = second
    if (length & 1) == 0 and second == (length - 2) // 2:
        second = 2 * (second + 1)
        v[first + hole] = v[first + second - 1]
        hole = second - 1
    parent = (hole - 1) // 2
    while hole > top and comp(v[first + parent], value):
        v[first + hole] = v[first + parent]
        hole = parent
        parent = (hole - 1) // 2
    v[first + hole] = value


def _heap_select(v, first, middle, last, comp):
    length = middle - first
    if length >= 2:
        parent = (length - 2) // 2
        while True:
            _adjust_heap(v, first, parent, length, v[first + parent], comp)
            if parent == 0:
                break
            parent -= 1
    for i in range(middle, last):
        if comp(v[i], v[first]):
            value = v[i]
            v[i] = v[first]
            _adjust_heap(v, first, 0, length, value, comp)


def nth_element(v, first, nth, last, comp):
    if first == last or nth == last:
        return
    depth_limit = 2 * ((last - first).bit_length() - 1)   # std::__lg(n) * 2
    while last - first > 3:
        if depth_limit == 0:
            _heap_select(v, first, nth + 1, last, comp)
            v[first], v[nth] = v[nth], v[first]
            return
        depth_limit -= 1
        mid = first + (last - first) // 2
        _move_median_to_first(v, first, first + 1, mid, last - 1, comp)
        cut = _unguarded_partition(v, first + 1, last, first, comp)
        if cut <= nth:
            first = cut
        else:
            last = cut
    _insertion_sort(v, first, last, comp)


# ------------------------------------------------------------------------------------------
# BVH_KDtree — bvh.cpp:5-93
# ------------------------------------------------------------------------------------------
def kd_tree(centers, bbs):
    n = len(centers)
    ids = list(range(n))
    splt = [0, n]
    d = 0
    depth = int(math.ceil(float(np.log2(F(n)))))   # int(ceilf(log2f(float(n))))
    for _ in range(1, depth):
        splt2 = [splt[0]]
        for i in range(1, len(splt)):
            j0, j2 = splt[i - 1], splt[i]
            j1 = (j0 + j2) // 2
            nth_element(ids, j0, j1, j2, lambda a, b, d=d: centers[a][d] < centers[b][d])
            splt2 += [j1, j2]
        splt = splt2
        d = (d + 1) % 3
    n_leaf = 1 << depth
    n_node = 2 * n_leaf - 1
    leaves = np.full(n_leaf, -1, np.int32)
    nodes = np.zeros((n_node, 6), F)
    j, k = n_node - 1, n_leaf - 1
    for i in range(len(splt) - 1, 0, -1):
        a = splt[i - 1]
        if splt[i] - a == 1:
            pid = ids[a]
            leaves[k], leaves[k - 1] = -1, pid
            nodes[j] = bbs[pid]
            nodes[j - 1] = bbs[pid]
        else:
            pid = ids[a + 1]
            leaves[k] = pid
            nodes[j] = bbs[pid]
            pid = ids[a]
            leaves[k - 1] = pid
            nodes[j - 1] = bbs[pid]
        k -= 2
        j -= 2
    k = n_node - 1
    while k >= 2:   # merge (scene.cpp:91-100), bottom up
        p = (k - 2) // 2
        nodes[p, :3] = np.minimum(nodes[k, :3], nodes[k - 1, :3])
        nodes[p, 3:] = np.maximum(nodes[k, 3:], nodes[k - 1, 3:])
        k -= 2
    return depth, nodes, leaves


# ------------------------------------------------------------------------------------------
# the reference scenes — montecarlo.cpp:33-46, 143-180, 629-795
# ------------------------------------------------------------------------------------------
ROUGE = (0.9, 0, 0, 1)
VERT = (0, 0.9, 0, 1)
BLEU = (0, 0, 0.9, 1)
JAUNE = (0.9, 0.9, 0, 1)
CYAN = (0, 0.9, 0.9, 1)
MAGENTA = (0.9, 0, 0.9, 1)
BLANC = (0.9, 0.9, 0.9, 1)
NOIR = (0, 0, 0, 1)


def OPA(c, o):
    c = list(np.asarray(c, F))
    c[3] = F(o)
    return c


def _menger(sc, m, d, s, mater):   # montecarlo.cpp:143-180
    x = F(F(2.0) / F(3.0))
    y = F(F(s) / F(3.0))
    offs = [(x, x, 0), (-x, x, 0), (-x, -x, 0), (x, -x, 0), (x, 0, x), (-x, 0, x), (-x, 0, -x), (x, 0, -x),
            (0, x, x), (0, -x, x), (0, -x, -x), (0, x, -x),
            (x, x, x), (-x, x, x), (-x, -x, x), (x, -x, x), (x, x, -x), (-x, x, -x), (-x, -x, -x), (x, -x, -x)]
    for o in offs:
        mm = mul(m, mul(translate(*o), scale(y)))
        if d > 0:
            _menger(sc, mm, d - 1, s, mater)
        else:
            sc.add_cube(mm, mater)


def build(scene_id: int, light_intensity: float = 1.2):
    """(prims, nodes, leaves, depth, nb_emissive) of reference scene 1..8 (keys Q..I)."""
    li = F(light_intensity)
    T, S, M, L = translate, scale, Material, Material.light
    sc = Scene()
    if scene_id == 1:   # scene_box_diffuse :701-717
        sc.add_orientedQuad(mul(T(0, 0, -100), S(100, 100, 1)), M(BLANC))
        sc.add_orientedQuad(mul(T(0, 0, 100), rotateX(180), S(100, 100, 1)), M(BLANC))
        sc.add_orientedQuad(mul(T(0, 100, 0), rotateX(90), S(100, 100, 1)), M(CYAN))
        sc.add_orientedQuad(mul(T(0, -100, 0), rotateX(-90), S(100, 100, 1)), M(JAUNE))
        sc.add_orientedQuad(mul(T(-100, 0, 0), rotateY(90), S(100, 100, 1)), M(ROUGE))
        sc.add_orientedQuad(mul(T(100, 0, 0), rotateY(-90), S(100, 100, 1)), M(VERT))
        sc.add_cube(mul(T(70, 20, -40), rotateZ(20), S(20, 20, 60)), M(BLANC))
        sc.add_cube(mul(T(-70, 40, -40), rotateZ(-20), S(20, 20, 60)), M(BLANC))
        sc.add_orientedQuad(mul(T(0, 0, 99), rotateX(180), S(40, 40, 1)), L(BLANC, F(F(10) * li)))
    elif scene_id == 2:   # scene_box_balls :720-741
        sc.add_orientedQuad(mul(T(0, 0, -100), S(100, 100, 1)), M(BLANC))
        sc.add_orientedQuad(mul(T(0, 0, 100), rotateX(180), S(100, 100, 1)), M(BLANC))
        sc.add_orientedQuad(mul(T(0, 100, 0), rotateX(90), S(100, 100, 1)), M(CYAN))
        sc.add_orientedQuad(mul(T(0, 99, 0), rotateX(90), S(40, 60, 1)), M(BLANC, 1, 1))
        sc.add_orientedQuad(mul(T(0, -100, 0), rotateX(-90), S(100, 100, 1)), M(BLANC))
        sc.add_orientedQuad(mul(T(-100, 0, 0), rotateY(90), S(100, 100, 1)), M(BLANC))
        sc.add_orientedQuad(mul(T(100, 0, 0), rotateY(-90), S(100, 100, 1)), M(BLANC))
        sc.add_cube(mul(T(70, 20, -60), rotateZ(20), S(20, 20, 40)), M(ROUGE))
        sc.add_cube(mul(T(-70, 40, -60), rotateZ(-20), S(20, 20, 40)), M(VERT))
        sc.add_sphere(mul(T(0, 50, -80), S(20)), M(MAGENTA, 0.8, 0.995))
        sc.add_sphere(mul(T(0, -30, 0), S(40)), M(OPA(JAUNE, 0.5), 0.65, 1))
        sc.add_sphere(mul(T(70, 20, 5), S(20)), M(OPA(ROUGE, 0.2), 0.8, 0.95))
        sc.add_sphere(mul(T(-70, 40, 5), S(20)), M(VERT, 0.7, 0.9))
        sc.add_orientedQuad(mul(T(0, 0, 99), rotateX(180), S(40, 40, 1)), L(BLANC, F(F(12.0) * li)))
    elif scene_id == 3:   # scene_menger :683-699
        sc.add_orientedQuad(mul(T(0, 0, -100), S(9000, 9000, 1)), M(BLANC, 0.8, 0.999))
        _menger(sc, mul(T(0, 0, -50), rotateZ(15), S(50)), 1, F(0.9), M(MAGENTA))
        sc.add_cylinder(mul(T(80, 80, -75), S(15, 15, 25)), M(BLEU))
        sc.add_cylinder(mul(T(-80, 80, -75), S(15, 15, 25)), M(VERT))
        sc.add_cylinder(mul(T(-80, -80, -75), S(15, 15, 25)), M(ROUGE))
        sc.add_cylinder(mul(T(80, -80, -75), S(15, 15, 25)), M(JAUNE))
        sc.add_sphere(mul(T(80, 80, -30), S(20)), M(CYAN, 0.6, 0.998))
        sc.add_sphere(mul(T(-80, 80, -30), S(20)), M(OPA(VERT, 0.1), 0.7, 0.5))
        sc.add_sphere(mul(T(-80, -80, -30), S(20)), M(ROUGE, 0.95, 0.97))
        sc.add_sphere(mul(T(80, -80, -30), S(20)), M(OPA(JAUNE, 0.25), 0.5, 0.999))
        sc.add_sphere(mul(T(0, 0, -50), S(20)), M(BLANC, 1, 1))
    elif scene_id == 4:   # scene_box_no_top :629-652
        sc.add_orientedQuad(mul(T(0, 0, -100), S(100, 100, 1)), M(BLANC))
        sc.add_orientedQuad(mul(T(0, 100, 0), rotateX(90), S(100, 100, 1)), M(CYAN))
        sc.add_orientedQuad(mul(T(0, 99, 0), rotateX(90), S(40, 60, 1)), M(BLANC, 1, 1))
        sc.add_orientedQuad(mul(T(0, -100, 0), rotateX(-90), S(100, 100, 1)), M(BLANC))
        sc.add_orientedQuad(mul(T(-100, 0, 0), rotateY(90), S(100, 100, 1)), M(BLANC))
        sc.add_orientedQuad(mul(T(100, 0, 0), rotateY(-90), S(100, 100, 1)), M(BLANC))
        sc.add_cube(mul(T(70, 20, -60), rotateZ(20), S(20, 20, 40)), M(ROUGE))
        sc.add_cube(mul(T(-70, 40, -60), rotateZ(-20), S(20, 20, 40)), M(VERT))
        sc.add_sphere(mul(T(0, 50, -80), S(20)), M(MAGENTA, 0.8, 0.995))
        sc.add_sphere(mul(T(0, -30, 0), S(40)), M(OPA(JAUNE, 0.1), 0.65, 1))
        sc.add_sphere(mul(T(70, 20, 5), S(20)), M(ROUGE, 0.8, 0.95))
        sc.add_sphere(mul(T(-70, 40, 5), S(20)), M(VERT, 0.7, 0.9))
        sc.add_orientedQuad(mul(T(99, -10, -40), rotateY(-90), S(60, 5, 1)), L(BLANC, F(F(10) * li)))
    elif scene_id == 5:   # scene_materials :743-753
        sc.add_cube(mul(T(0, 0, -50), S(9000, 9000, 1)), M(BLANC))
        for j in range(-5, 6):
            for i in range(-5, 6):
                # Material(ROUGE, 1.0f-0.075*(i+5), 1.0f-0.01f*(j+5)): the shininess in binary64
                # (a double literal), then cast; the roughness in binary32
                shin = F(1.0 - 0.075 * (i + 5))
                rough = F(F(1.0) - F(F(0.01) * F(j + 5)))
                sc.add_sphere(mul(T(30 * i, 30 * j, -41), S(8)), M(ROUGE, shin, rough))
    elif scene_id == 6:   # scene_4boules :756-770
        sc.add_cube(mul(T(0, 0, -51), S(9000, 9000, 1)), M(BLANC, 0.2, 0.99999))
        sc.add_sphere(mul(T(110, 0, 0), S(50)), M(OPA(MAGENTA, 0.01), 0.7, 0.99))
        sc.add_sphere(mul(T(-110, 0, 0), S(50)), M(OPA(ROUGE, 0.15), 0.5, 0.5))
        sc.add_sphere(mul(T(0, 110, 0), S(50)), M(OPA(CYAN, 0.05), 0.8, 0.7))
        sc.add_sphere(mul(T(0, -110, 0), S(50)), M(OPA(VERT, 0.25), 0.7, 0.9))
        sc.add_orientedQuad(mul(T(200, 0, 100), rotateY(-110), S(20, 20, 1)), L(BLANC, F(F(20) * li)))
    elif scene_id == 7:   # scene_menger_lights :655-681
        sc.add_cube(mul(T(0, 0, -10), S(9975, 9975, 1)), M(BLANC, 0.5, 0.9))
        _menger(sc, mul(T(0, 0, 42), rotateZ(15), S(50.0)), 1, F(0.9), M(ROUGE))
        _menger(sc, mul(T(-105, 0, 11), S(20.0)), 0, F(0.7), M(BLEU))
        _menger(sc, mul(T(0, -105, 11), S(20.0)), 0, F(0.7), M(CYAN))
        _menger(sc, mul(T(0, 105, 11), S(20.0)), 0, F(0.7), M(MAGENTA))
        _menger(sc, mul(T(105, 0, 11), S(20.0)), 0, F(0.7), M(JAUNE))
        sc.add_sphere(mul(T(-100, -100, 5), S(15)), M((1, 1, 1, 0.3), 0.99, 0.6))
        sc.add_sphere(mul(T(-100, 100, 5), S(15)), M((1, 0, 1, 0.2), 0.8, 0.4))
        sc.add_sphere(mul(T(100, 100, 5), S(15)), M((1, 1, 0, 0.4), 0.6, 0.2))
        sc.add_sphere(mul(T(100, -100, 5), S(15)), M((0, 1, 0, 0.1), 0.4, 0.1))
        sc.add_cube(mul(T(0, 0, 500), S(1000, 1000, 1)), M(NOIR))
        for t, r in (((0, 0, 42), 10), ((-105, 0, 11), 5), ((105, 0, 11), 5), ((0, 105, 11), 5), ((0, -105, 11), 5)):
            sc.add_sphere(mul(T(*t), S(r)), L(BLANC, F(F(10) * li)))
    elif scene_id == 8:   # scene_colonnes :772-795
        # 0.6f*BLANC + 0.4f*VERT: binary32 vector arithmetic
        ground = [F(F(F(0.6) * F(a)) + F(F(0.4) * F(b))) for a, b in zip(BLANC, VERT)]
        sc.add_orientedQuad(mul(T(0, 0, -100), S(90000, 90000, 1)), M(ground, 0.7, 0.9999))
        for i in range(-1000, 1001, 250):
            for j in range(-1000, 1001, 250):
                sc.add_cylinder(mul(T(i, j, -98), S(60, 60, 2)), M(BLANC))
                sc.add_cylinder(mul(T(i, j, -93), S(50, 50, 3)), M(BLANC))
                sc.add_cylinder(mul(T(i, j, -85), S(30, 30, 5)), M(BLANC))
                sc.add_cylinder(mul(T(i, j, 0), S(20, 20, 80)), M(BLANC))
                sc.add_cube(mul(T(i, j, 90), S(30, 30, 10)), M(BLANC))
                for a in (45, 135, 225, 315):
                    sc.add_cube(mul(T(i, j, 105), rotateZ(a), T(90, 0, 0), S(80, 10, 5)), M(BLANC))
                sc.add_cylinder(mul(T(i + 125, j + 125, 115), S(75, 75, 5)), M(BLANC))
                sc.add_cylinder(mul(T(i, j, 115), S(65, 65, 5)), M(BLANC))
        sc.add_sphere(mul(T(150, 375, -70), S(30)), M(JAUNE, 0.5, 0.999))
        sc.add_sphere(mul(T(100, 125, -70), S(30)), M(OPA(CYAN, 0.2), 0.5, 0.9))
        sc.add_cube(mul(T(125, -125, -80), rotateZ(45), S(20)), M(ROUGE, 0.1, 0.2))
    else:
        raise ValueError(f"scene {scene_id}: 1..8")
    return sc.finalize()


def custom(ops):
    """A scene of (type, column-major transform, material (r, g, b, a, shin, rough, emi)) records
    through the same producer (the analogue of the oracle's custom_scene)."""
    sc = Scene()
    add = {1: sc.add_sphere, 2: sc.add_cube, 3: sc.add_cylinder, 4: sc.add_cone, 5: sc.add_orientedQuad}
    for t, m16, mat in ops:
        m16 = np.asarray(m16, F)
        mat = np.asarray(mat, F)
        add[int(t)](m16.reshape(4, 4).T.copy(), Material(mat[:4], mat[4], mat[5], mat[6]))
    return sc.finalize()


# ------------------------------------------------------------------------------------------
# the canonical camera — camera.cpp:28-95, camera.h:62-93, montecarlo.cpp:389, 404-405, 439-440
# ------------------------------------------------------------------------------------------
def camera(W: int, H: int):
    """(invPV, invV), 16 f32 column-major each, for a W x H viewport: fov 0.78, scene radius 145,
    frame identity, pivot 0; GLViewer::get_projection_matrix / get_modelview_matrix cast the
    binary64 matrices to binary32; view = MV * rotateX(-80); invPV = (P * view)^-1, invV = view^-1."""
    fov, radius = 0.78, 145.0
    focal = radius / math.tan(fov / 2.0)
    asp = float(W) / float(H)
    d = focal - 0.0                       # frame translation z = 0
    zn, zf = max(0.01, d - radius), d + radius
    ri = 1.0 / (zn - zf)
    f = 1.0 / math.tan(fov / 2.0)
    m0, m5 = (f / asp, f) if asp > 1 else (f, f * asp)
    P = np.zeros((4, 4), F)
    P[0, 0], P[1, 1] = F(m0), F(m5)
    P[2, 2], P[2, 3], P[3, 2] = F((zn + zf) * ri), F(2 * zn * zf * ri), F(-1.0)
    MV = ident()
    MV[2, 3] = F(-focal)
    view = mul(MV, rotateX(-80))
    return colmajor(inverse(mul(P, view))), colmajor(inverse(view))
