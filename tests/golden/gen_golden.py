#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (committed; rerun to regenerate).

1. kat.npz — known-answer vectors from an INDEPENDENT numpy float32 restatement of the
   pieces of the sampling loop (RNG, transcendental contract, hemisphere sampler,
   primitive intersections), written from the GLSL text (raytracer_func.frag,
   tp/montecarlo.frag) and DESIGN.md §3, not from oracle.cpp.  fma is emulated exactly
   (double product + TwoSum + midpoint fix-up), so the vectors are bit-exact.
2. img_s{scene}_v{variant}.npy — small accumulator images rendered by the C++ oracle
   (regression pins for the oracle and direct fixtures for the GPU tests) on scene buffers and
   cameras from scene_restate.py.
3. paths.npz (`python gen_golden.py paths`) — 688 whole samples of the integrator
   ((pixel, pass) at 1080p on all eight reference scenes, 6 and 5 also at IOR 1.5, and a scene
   with the pure refraction branch; 96 of them run montecarlo_mat / montecarlo_mat_tr) from the
   same independent numpy restatement extended to the camera
   ray, the BVH DFS, intersection_info and random_path, with the branch sequence each took; the
   scene buffers, BVHs and cameras come from scene_restate.py, a numpy restatement of the host
   producer (Transfo, PrimData, prim_bb, sortEmissiveFirst, libstdc++ nth_element, BVH_KDtree,
   camera), so nothing of the fixture comes from oracle.cpp (round 5).

The reference itself cannot run here (no GL 4.3 / Eigen / GLFW / assimp):
parity with the executed GLSL is unpinned; these fixtures pin the restatement.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
import scene_restate  # noqa: E402  (numpy restatement of the host producer and camera)

f32 = np.float32
u32 = np.uint32


# ----------------------------------------------------------------------------------
# exact binary32 fma in numpy
# ----------------------------------------------------------------------------------
def fma32(a, b, c):
    """round-to-nearest-even binary32 of a*b+c, exactly (no double-rounding)."""
    a = np.asarray(a, np.float32).astype(np.float64)
    b = np.asarray(b, np.float32).astype(np.float64)
    c = np.asarray(c, np.float32).astype(np.float64)
    p = a * b                            # exact: 24+24 significant bits
    s = p + c
    bb = s - p
    err = (p - (s - bb)) + (c - bb)      # TwoSum: s + err == p + c exactly
    r = s.astype(np.float32)
    r64 = r.astype(np.float64)
    other = np.nextafter(r, np.where(s > r64, np.float32(np.inf), np.float32(-np.inf)).astype(np.float32))
    mid = (r64 + other.astype(np.float64)) * 0.5
    # float32(s) is correct unless s sits exactly on a binary32 midpoint and err != 0
    is_mid = (s != r64) & (s == mid) & (err != 0)
    res = np.where(is_mid, np.where(err > 0, np.maximum(r, other), np.minimum(r, other)), r)
    return res.astype(np.float32) if np.ndim(res) else np.float32(res)


def dot3(a, b):
    return fma32(a[2], b[2], fma32(a[1], b[1], f32(a[0] * b[0])))


def normalize(v):
    r = f32(f32(1.0) / np.sqrt(dot3(v, v)))
    return [f32(v[0] * r), f32(v[1] * r), f32(v[2] * r)]


def length(v):
    return f32(np.sqrt(dot3(v, v)))


def cross(a, b):
    return [f32(a[1] * b[2] - a[2] * b[1]), f32(a[2] * b[0] - a[0] * b[2]), f32(a[0] * b[1] - a[1] * b[0])]


def vsub(a, b):
    return [f32(a[i] - b[i]) for i in range(3)]


def vadd(a, b):
    return [f32(a[i] + b[i]) for i in range(3)]


def vmul(a, s):
    return [f32(a[i] * s) for i in range(3)]


def xpoint(m, p):   # column-major mat4, rows 0..2, fma chain x,y,z then + translation
    return [f32(fma32(m[8 + r], p[2], fma32(m[4 + r], p[1], f32(m[r] * p[0]))) + m[12 + r]) for r in range(3)]


def xdir(m, d):
    return [fma32(m[8 + r], d[2], fma32(m[4 + r], d[1], f32(m[r] * d[0]))) for r in range(3)]


# ----------------------------------------------------------------------------------
# RNG (raytracer_func.frag:90-135)
# ----------------------------------------------------------------------------------
def xxhash32(px, py, pz):
    with np.errstate(over="ignore"):
        px, py, pz = u32(px), u32(py), u32(pz)
        P2, P3, P4, P5 = u32(2246822519), u32(3266489917), u32(668265263), u32(374761393)
        h = u32(pz + P5 + px * P3)
        h = u32(P4 * u32((h << u32(17)) | (h >> u32(15))))
        h = u32(h + py * P3)
        h = u32(P4 * u32((h << u32(17)) | (h >> u32(15))))
        h = u32(P2 * u32(h ^ (h >> u32(15))))
        h = u32(P3 * u32(h ^ (h >> u32(13))))
        return u32(h ^ (h >> u32(16)))


def srand(tcx, tcy, npass, date):
    f = f32(1 + npass)
    mid = f32(f32(f32(npass) * f32(3.14)) + f32(date))
    w = [f32(f32(f32(tcx) * f) * f32(1.125)), f32(f32(mid * f) * f32(1.125)), f32(f32(f32(tcy) * f) * f32(1.125))]
    return [int(np.array(x, np.float32).view(np.uint32)) for x in w]


def random_float(seed):
    m = int(xxhash32(*seed))
    v = np.array((m & 0x7FFFFF) | 0x3F800000, np.uint32).view(np.float32)
    seed[0] = (seed[0] + 11) & 0xFFFFFFFF
    seed[1] = (seed[1] + 43) & 0xFFFFFFFF
    seed[2] = (seed[2] + 67) & 0xFFFFFFFF
    return f32(v - f32(1.0))


# ----------------------------------------------------------------------------------
# transcendental contract
# ----------------------------------------------------------------------------------
def mc_sincos(x):
    x = f32(x)
    qf = f32(np.floor(f32(f32(x * f32(0.636619746685028076)) + f32(0.5))))
    q = int(qf)
    r = fma32(-qf, f32(1.57079637050628662), x)
    r = fma32(-qf, f32(-4.37113900018624283e-8), r)
    r = fma32(-qf, f32(-1.71512451e-15), r)
    s = f32(r * r)
    sp = fma32(fma32(f32(-1.9515295891e-4), s, f32(8.3321608736e-3)), s, f32(-1.6666654611e-1))
    sn = fma32(f32(r * s), sp, r)
    cp = fma32(fma32(f32(2.443315711809948e-5), s, f32(-1.388731625493765e-3)), s, f32(4.166664568298827e-2))
    cs = fma32(f32(s * s), cp, fma32(f32(-0.5), s, f32(1.0)))
    return [(sn, cs), (cs, f32(-sn)), (f32(-sn), f32(-cs)), (f32(-cs), sn)][q & 3]


LOG_P = [7.0376836292e-2, -1.1514610310e-1, 1.1676998740e-1, -1.2420140846e-1, 1.4249322787e-1,
         -1.6668057665e-1, 2.0000714765e-1, -2.4999993993e-1, 3.3333331174e-1]


def mc_log(x):
    x = f32(x)
    if not (x > 0):
        return f32(-np.inf) if x == 0 else f32(np.nan)
    if np.isinf(x):
        return x
    b = int(np.array(x, np.float32).view(np.uint32))
    e = 0
    if b < 0x00800000:
        x = f32(x * f32(8388608.0))
        b = int(np.array(x, np.float32).view(np.uint32))
        e = -23
    e += (b >> 23) - 127
    m = np.array((b & 0x7FFFFF) | 0x3F800000, np.uint32).view(np.float32)[()]
    if m > f32(1.41421353816986084):
        m = f32(m * f32(0.5))
        e += 1
    f = f32(m - f32(1.0))
    z = f32(f * f)
    p = f32(LOG_P[0])
    for c in LOG_P[1:]:
        p = fma32(p, f, f32(c))
    ef = f32(e)
    y = f32(f32(f * z) * p)
    y = fma32(ef, f32(-2.12194440e-4), y)
    y = fma32(f32(-0.5), z, y)
    r = f32(f + y)
    return fma32(ef, f32(0.693359375), r)


EXP2_P = [1.535336188319500e-4, 1.339887440266574e-3, 9.618437357674640e-3, 5.550332471162809e-2,
          2.402264791363012e-1, 6.931472028550421e-1]


def mc_exp2(x):
    x = f32(x)
    if np.isnan(x):
        return x
    if x >= 128:
        return f32(np.inf)
    if x < -150:
        return f32(0.0)
    kf = f32(np.floor(f32(x + f32(0.5))))
    f = f32(x - kf)
    p = f32(EXP2_P[0])
    for c in EXP2_P[1:]:
        p = fma32(p, f, f32(c))
    r = fma32(p, f, f32(1.0))
    k = int(kf)
    if k >= -126:
        return f32(r * np.array((k + 127) << 23, np.uint32).view(np.float32)[()])
    sc = np.array((k + 127 + 64) << 23, np.uint32).view(np.float32)[()]
    return f32(f32(r * sc) * f32(5.42101086242752217e-20))


def mc_pow(x, y):
    return mc_exp2(f32(f32(y) * f32(mc_log(x) * f32(1.44269502162933350))))


# ----------------------------------------------------------------------------------
# sampler (tp/montecarlo.frag:49-89)
# ----------------------------------------------------------------------------------
PI = f32(3.14159274101257324)


def random_ray(seed, D, rough):
    D = [f32(d) for d in D]
    W = normalize([D[0], f32(D[1] + f32(5.0)), f32(D[2] + f32(3.0))])
    U = normalize(cross(D, W))
    V = normalize(cross(D, U))
    alpha = f32(f32(rough) * f32(rough))
    beta = f32(f32(f32(2.0) * PI) * random_float(seed))
    t2 = f32(f32(-alpha * alpha) * mc_log(f32(f32(1.0) - random_float(seed))))
    ct = f32(f32(1.0) / np.sqrt(f32(f32(1.0) + t2)))
    one_m = f32(f32(1.0) - f32(ct * ct))
    st = f32(np.sqrt(one_m if (f32(0.0) < one_m) else f32(0.0)))   # GLSL max(0, x)
    sb, cb = mc_sincos(beta)
    sm = normalize([f32(cb * st), f32(sb * st), ct])
    m = [fma32(D[i], sm[2], fma32(V[i], sm[1], f32(U[i] * sm[0]))) for i in range(3)]
    return normalize(m)


# ----------------------------------------------------------------------------------
# primitive intersection (raytracer_func.frag:398-705), world-space distances
# ----------------------------------------------------------------------------------
EPS = f32(1e-10)
FMAX = f32(3.402823e38)


def intersect_prim(rec, Ow, Dw, best=None, index=0):
    """intersect_prim :681-705 on one primitive record; `best` is the closest_intersection
    record shared along a traversal (a fresh one when None)."""
    rec = np.asarray(rec, np.float32)
    t = int(rec[48])
    inv, trf = rec[16:32], rec[0:16]
    O = xpoint(inv, Ow)
    D = normalize(xdir(inv, Dw))
    if best is None:
        best = {"shape": -1, "dist": FMAX, "dir": -1, "pl": [f32(0)] * 3, "pg": [f32(0)] * 3, "index": -1}

    def cand(a, shape, d):
        Pl = vadd(O, vmul(D, a))
        Pg = xpoint(trf, Pl)
        dist = length(vsub([f32(v) for v in Ow], Pg))
        if dist < best["dist"]:
            best.update(shape=shape, dist=dist, dir=d, pl=Pl, pg=Pg, index=index)

    if t == 1:
        OO, OD, D2 = dot3(O, O), dot3(O, D), dot3(D, D)
        d4 = f32(f32(OD * OD) - f32(D2 * f32(OO - f32(1.0))))
        if d4 > 0:
            sq = f32(np.sqrt(d4))
            for a in (f32(-f32(OD + sq) / D2), f32(-f32(OD - sq) / D2)):
                if a > EPS:
                    cand(a, 1, 0)
    elif t == 5:
        if D[2] > -EPS:
            return best
        a = f32(-O[2] / D[2])
        Pl = vadd(O, vmul(D, a))
        if abs(Pl[0]) > 1 or abs(Pl[1]) > 1:
            return best
        cand(a, 5, 0)
    elif t == 2:
        al, cl = FMAX, 0
        for fc in range(6):
            c0 = fc // 2
            if abs(D[c0]) > EPS:
                c1, c2 = (c0 + 1) % 3, (c0 + 2) % 3
                cd = f32(-1.0 + 2.0 * (fc % 2))
                a = f32(f32(cd - O[c0]) / D[c0])
                if a > EPS and abs(f32(O[c1] + f32(a * D[c1]))) <= 1 and abs(f32(O[c2] + f32(a * D[c2]))) <= 1:
                    if a < al:
                        al, cl = a, fc
        if al < FMAX:
            cand(al, 2, cl)
    elif t == 3:
        cl, al = -1, FMAX
        if abs(D[2]) > EPS:
            for cd, code in ((f32(-1.0), 0), (f32(1.0), 1)):
                a = f32(f32(cd - O[2]) / D[2])
                if a > EPS:
                    rx, ry = f32(O[0] + f32(a * D[0])), f32(O[1] + f32(a * D[1]))
                    if fma32(ry, ry, f32(rx * rx)) < 1 and a < al:
                        cl, al = code, a
        O2 = fma32(O[1], O[1], f32(O[0] * O[0]))
        OD = fma32(O[1], D[1], f32(O[0] * D[0]))
        D2 = fma32(D[1], D[1], f32(D[0] * D[0]))
        d4 = f32(f32(OD * OD) - f32(D2 * f32(O2 - f32(1.0))))
        if d4 > 0:
            a = f32(-f32(OD + f32(np.sqrt(d4))) / D2)
            if a > EPS and a < al:
                z = f32(O[2] + f32(a * D[2]))
                if abs(z) < 1:
                    cl, al = 2, a
        if al < FMAX:
            cand(al, 3, cl)
    elif t == 4:   # Cone_intersect :579-640 (backward roots accepted: no a > EPS check)
        cl, tl = -1, FMAX
        if abs(D[2]) > EPS:
            t0 = f32(f32(f32(-1.0) - O[2]) / D[2])
            if t0 > EPS:
                rx, ry = f32(O[0] + f32(t0 * D[0])), f32(O[1] + f32(t0 * D[1]))
                if fma32(ry, ry, f32(rx * rx)) < 1 and t0 < tl:
                    cl, tl = 0, t0
        co = [O[0], O[1], f32(O[2] - f32(1.0))]
        a = f32(f32(D[2] * D[2]) - f32(0.8))
        b = f32(f32(2.0) * f32(f32(D[2] * co[2]) - f32(dot3(D, co) * f32(0.8))))
        c = f32(f32(co[2] * co[2]) - f32(dot3(co, co) * f32(0.8)))
        det = f32(f32(b * b) - f32(f32(f32(4.0) * a) * c))
        if det > 0:
            det = f32(np.sqrt(det))
            t1 = f32(f32(-b - det) / f32(f32(2.0) * a))
            if abs(f32(O[2] + f32(t1 * D[2]))) > 1:
                t1 = FMAX
            t2 = f32(f32(-b + det) / f32(f32(2.0) * a))
            if abs(f32(O[2] + f32(t2 * D[2]))) > 1:
                t2 = FMAX
            tt = t2 if t2 < t1 else t1          # GLSL min
            if tt < tl:
                cl, tl = 2, tt
        if tl < FMAX:
            cand(tl, 4, cl)
    return best


# ----------------------------------------------------------------------------------
# one whole sample of the integrator, for the path KATs (paths.npz): the camera ray
# (shaders/raytracer.vert:9-22 + strip interpolation), intersect_bvh's DFS
# (raytracer_func.frag:734-769) with intersect_bv (:314-352), intersection_info (:812-897)
# and random_path (tp/montecarlo.frag:100-179), written from the GLSL text and the
# arithmetic contract of DESIGN.md §3 (binary32 round-to-nearest, no contraction except the
# fma chains of dot / mat·vec, box-test divisions as correctly rounded reciprocals hoisted to
# node upload and ray set-up, GLSL builtins by their definitions) — not from oracle.cpp.
# ----------------------------------------------------------------------------------
BIAS = f32(1e-2)


def rcp(x):
    return f32(f32(1.0) / f32(x))


def glsl_mix(x, y, a):                       # x·(1−a) + y·a
    return f32(f32(f32(x) * f32(f32(1.0) - f32(a))) + f32(f32(y) * f32(a)))


def glsl_reflect(I, N):                      # I − 2·dot(N,I)·N
    d2 = f32(f32(2.0) * dot3(N, I))
    return [f32(I[k] - f32(d2 * N[k])) for k in range(3)]


def glsl_refract(I, N, eta):                 # GLSL 4.30 §8.5
    eta = f32(eta)
    d = dot3(N, I)
    k = f32(f32(1.0) - f32(f32(eta * eta) * f32(f32(1.0) - f32(d * d))))
    if k < 0:
        return [f32(0.0)] * 3
    t = f32(f32(eta * d) + f32(np.sqrt(k)))
    return [f32(f32(eta * I[c]) - f32(t * N[c])) for c in range(3)]


def r_schlick(ior, I, N):                    # tp/montecarlo.frag:91-98
    ior = f32(ior)
    r0 = f32(f32(ior - f32(1.0)) / f32(ior + f32(1.0)))
    r0 = f32(r0 * r0)
    x = f32(f32(1.0) - dot3(N, I))
    v = f32(f32(1.0) - r0)
    for _ in range(5):
        v = f32(v * x)
    v = f32(r0 + v)
    return min(max(v, f32(0.0)), f32(1.0))


def node_boxes(nodes):
    """intersect_bv's centre and half-width (bbmin+bbmax)/2, 0.5·(bbmax−bbmin) per node, and the
    hoisted 1/half-width (contract §3.5)."""
    out = []
    for b in np.asarray(nodes, np.float32).reshape(-1, 6):
        c = [f32(f32(b[k] + b[3 + k]) / f32(2.0)) for k in range(3)]
        w = [f32(f32(0.5) * f32(b[3 + k] - b[k])) for k in range(3)]
        with np.errstate(divide="ignore"):
            iw = [rcp(v) for v in w]
        out.append((c, w, iw))
    return out


def intersect_bv(box, O, D, invD, closest_dist):
    c, w, iw = box
    with np.errstate(invalid="ignore", over="ignore"):
        Oi = [f32(f32(O[k] - c[k]) * iw[k]) for k in range(3)]
        Di = [f32(D[k] * iw[k]) for k in range(3)]
        if all(abs(Oi[k]) < 1 for k in range(3)):
            return True
        al = FMAX
        for fc in range(6):
            c0 = fc // 2
            if abs(Di[c0]) > EPS:
                c1, c2 = (c0 + 1) % 3, (c0 + 2) % 3
                cd = f32(-1.0 + 2.0 * (fc % 2))
                a = f32(f32(cd - Oi[c0]) * f32(invD[c0] * w[c0]))      # (cd − Oi)/Di
                if a > EPS and abs(f32(Oi[c1] + f32(a * Di[c1]))) <= 1 and abs(f32(Oi[c2] + f32(a * Di[c2]))) <= 1:
                    if a < al:
                        al = a
        if al < FMAX:
            Pg = [f32(f32(f32(f32(al * Di[k]) + Oi[k]) * w[k]) + c[k]) for k in range(3)]
            return length(vsub(O, Pg)) <= closest_dist
    return False


def intersect_bvh(prims, boxes, leaves, depth, O, D, stats=None):
    """traverse_all_bvh: the literal stack of :734-769 (right child popped first)."""
    best = {"shape": -1, "dist": FMAX, "dir": -1, "pl": [f32(0)] * 3, "pg": [f32(0)] * 3, "index": -1}
    with np.errstate(divide="ignore"):
        invD = [rcp(D[k]) for k in range(3)]
    max_line = 2 ** depth - 1
    stack = [0]
    while stack:
        i = stack.pop()
        if i >= max_line:
            p = int(leaves[i - max_line])
            if p >= 0:
                if int(prims[p][48]) not in (1, 2, 3, 5):
                    raise NotImplementedError("path KATs cover sphere / cube / cylinder / quad scenes")
                intersect_prim(prims[p], O, D, best, p)
        else:
            if stats is not None:
                stats["node"] += 1
            j = 2 * i + 1
            if intersect_bv(boxes[j], O, D, invD, best["dist"]):
                stack.append(j)
            j += 1
            if intersect_bv(boxes[j], O, D, invD, best["dist"]):
                stack.append(j)
    return best


def intersection_info(prims, hit):
    rec = prims[hit["index"]]
    pl, Pg, sh, d = hit["pl"], hit["pg"], hit["shape"], hit["dir"]
    if sh == 1:
        q = [f32(f32(2.0) * pl[k]) for k in range(3)]
    elif sh == 2:
        No = [f32(0.0)] * 3
        No[d // 2] = f32(1.0) if d % 2 != 0 else f32(-1.0)
        q = vadd(pl, No)
    elif sh == 3:
        No = [f32(0.0), f32(0.0), f32(1.0) if d % 2 != 0 else f32(-1.0)] if d < 2 else [pl[0], pl[1], f32(0.0)]
        q = vadd(pl, No)
    elif sh == 5:
        q = vadd(pl, [f32(0.0), f32(0.0), f32(1.0)])
    else:
        raise NotImplementedError(sh)
    return normalize(vsub(xpoint(rec[0:16], q), Pg)), Pg


def camera_dir(invPV, invV, W, H, x, y):
    """raytracer.vert corner rays, the strip's barycentric interpolation at screen_tc, and
    raytrace's normalize (montecarlo.frag:182-188).  Returns (Ori, D, u, v)."""
    def mv4(m, v):     # mat4 · vec4, fma chain x, y, z, w
        return [fma32(m[12 + r], v[3], fma32(m[8 + r], v[2], fma32(m[4 + r], v[1], f32(m[r] * v[0]))))
                for r in range(4)]
    P4 = mv4(invV, [f32(0), f32(0), f32(0), f32(1)])
    Ori = P4[:3]
    corners = []
    for vid in range(4):
        tc = [f32(vid % 2), f32(vid // 2)]
        cc = [f32(f32(2.0) * tc[0] - f32(1.0)), f32(f32(2.0) * tc[1] - f32(1.0))]
        Q = mv4(invPV, [cc[0], cc[1], f32(1), f32(1)])
        corners.append(normalize([f32(f32(Q[k] / Q[3]) - Ori[k]) for k in range(3)]))
    u = f32(f32(f32(x) + f32(0.5)) / f32(W))
    v = f32(f32(f32(y) + f32(0.5)) / f32(H))
    if f32(u + v) <= 1:
        w0 = f32(f32(f32(1.0) - u) - v)
        d = [f32(f32(f32(corners[0][k] * w0) + f32(corners[1][k] * u)) + f32(corners[2][k] * v)) for k in range(3)]
    else:
        w1, w3, w2 = f32(f32(1.0) - v), f32(f32(u + v) - f32(1.0)), f32(f32(1.0) - u)
        d = [f32(f32(f32(corners[1][k] * w1) + f32(corners[3][k] * w3)) + f32(corners[2][k] * w2)) for k in range(3)]
    return Ori, normalize(d), u, v


def random_path(prims, boxes, leaves, depth, seed, D, O, B, ior):
    """tp/montecarlo.frag:100-179 as written.  Returns (rgb, branch codes taken): S sky,
    E emissive end, R reflect, T pure refraction, M/m mixed reflect/refract, F diffuse,
    X budget exhausted (black), I an inner traversal that missed (N, P unchanged)."""
    trace = []
    total = [f32(0.0)] * 3
    stack = [(O, D, [f32(0.8)] * 3)]
    i = 0
    while i < B and stack:
        O, D, att = stack.pop()
        hit = intersect_bvh(prims, boxes, leaves, depth, O, D)
        if hit["shape"] < 0:
            a = max(f32(0.0), D[2])
            sky = [glsl_mix(f32(0.5), f32(1.0), a), glsl_mix(f32(0.5), f32(1.0), a), glsl_mix(f32(0.9), f32(0.8), a)]
            trace.append("S")
            return [f32(total[k] + f32(att[k] * sky[k])) for k in range(3)], trace
        N, P = intersection_info(prims, hit)
        rec = prims[hit["index"]]
        col, mat = rec[52:56], rec[56:60]
        ray = random_ray(seed, N, f32(f32(1.0) - mat[1]))
        rs = r_schlick(ior, D, N)
        R = glsl_reflect([f32(-r) for r in ray], N)
        E = normalize(vsub(O, P))
        se = glsl_mix(f32(100.0), f32(2.0), mat[1])
        spec = mc_pow(max(f32(0.0), dot3(E, R)), se)
        total = [f32(total[k] + f32(f32(col[k] * f32(0.1)) +
                                    f32(f32(f32(att[k] * mat[2]) * f32(f32(1.0) - mat[0])) * col[3]))) for k in range(3)]
        if mat[2] <= 0.5 and len(stack) < 9:
            mx = [glsl_mix(att[k], col[k], mat[0]) for k in range(3)]

            def reflect_push():
                na = [f32(f32(col[k] * att[k]) + f32(f32(f32(f32(att[k] * col[3]) * rs) * spec) * mx[k]))
                      for k in range(3)]
                rd = random_ray(seed, glsl_reflect(D, N), f32(f32(1.0) - f32(mat[0] * mat[1])))
                stack.append(([f32(P[k] + f32(BIAS * N[k])) for k in range(3)], rd, na))

            def refract_push(Din):
                na = [f32(f32(col[k] * att[k]) +
                          f32(f32(f32(f32(att[k] * f32(f32(1.0) - col[3])) * f32(f32(1.0) - rs)) * spec) * mx[k]))
                      for k in range(3)]
                Oin = [f32(P[k] - f32(BIAS * N[k])) for k in range(3)]
                inner = intersect_bvh(prims, boxes, leaves, depth, Oin, Din)
                N2, P2 = N, P
                if inner["shape"] >= 0:
                    N2, P2 = intersection_info(prims, inner)
                else:
                    trace.append("I")          # intersection_info leaves N, P as they were
                out = glsl_refract(Din, [f32(-n) for n in N2], f32(f32(1.0) / f32(ior)))
                stack.append(([f32(P2[k] + f32(BIAS * N2[k])) for k in range(3)], out, na))

            if mat[0] > 0 and col[3] == 1:
                trace.append("R")
                reflect_push()
            elif col[3] < 1 and mat[0] == 0:
                trace.append("T")
                refract_push(glsl_refract(D, N, ior))
            elif col[3] < 1 and mat[0] > 0:
                if random_float(seed) > 0.5:
                    trace.append("M")
                    reflect_push()
                else:
                    trace.append("m")
                    refract_push(D)                # the mixed branch does not refract on entry
            else:
                trace.append("F")
                stack.append(([f32(P[k] + f32(BIAS * N[k])) for k in range(3)], ray,
                              [f32(f32(col[k] * att[k]) + f32(f32(att[k] * spec) * mx[k])) for k in range(3)]))
        else:
            trace.append("E")
            return total, trace
        i += 1
    trace.append("X")
    return [f32(0.0)] * 3, trace


def variant_path(prims, boxes, leaves, depth, seed, D, O, variant):
    """tp/montecarlo_mat.frag:5-20 (variant 1) / tp/montecarlo_mat_tr.frag:5-20 (variant 2): one
    traversal; a miss is (0, 0, 0.2); a hit returns abs(N) * random_vec3() (three draws, x then
    y then z: GLSL evaluates constructor arguments left to right) or col.rgb * random_float()."""
    hit = intersect_bvh(prims, boxes, leaves, depth, O, D)
    if hit["shape"] < 0:
        return [f32(0.0), f32(0.0), f32(0.2)], ["S"]
    N, _ = intersection_info(prims, hit)
    col = prims[hit["index"]][52:56]
    if variant == 1:
        r = [random_float(seed) for _ in range(3)]
        return [f32(f32(abs(N[k])) * r[k]) for k in range(3)], ["V"]
    r = random_float(seed)
    return [f32(col[k] * r) for k in range(3)], ["V"]


def sample(prims, nodes, leaves, depth, invPV, invV, W, H, x, y, npass, B, ior, date=0.0, variant=0):
    """One (pixel, pass) sample of montecarlo.frag (or a variant): srand at screen_tc, then
    random_path."""
    Ori, D, u, v = camera_dir(invPV, invV, W, H, x, y)
    seed = srand(u, v, npass, f32(date))
    if variant:
        return variant_path(prims, node_boxes(nodes), leaves, depth, seed, D, Ori, variant)
    return random_path(prims, node_boxes(nodes), leaves, depth, seed, D, Ori, B, ior)


# ----------------------------------------------------------------------------------
def make_kat(rng: np.random.Generator):
    kat = {}
    # xxhash32 on random triples
    xs = rng.integers(0, 2**32, size=(256, 3), dtype=np.uint64).astype(np.uint32)
    kat["xx_in"] = xs
    kat["xx_out"] = np.array([xxhash32(*x) for x in xs], np.uint32)
    # srand + 16 random floats for pixels/passes
    cases = [(0.5 / 64, 0.5 / 48, 1, 0.0), (0.9921875, 0.0104166670, 7, 0.0), (0.3, 0.7, 256, 0.0),
             (0.00026041666, 0.99953705, 84000, 0.0), (0.5, 0.5, 1, 0.016), (0.125, 0.875, 33, 0.0)]
    kat["srand_in"] = np.array([c[:2] for c in cases], np.float32)
    kat["srand_pass"] = np.array([c[2] for c in cases], np.int32)
    kat["srand_date"] = np.array([c[3] for c in cases], np.float32)
    seeds, seqs = [], []
    for (tx, ty, p, d) in cases:
        s = srand(f32(tx), f32(ty), p, f32(d))
        seeds.append(list(s))
        seqs.append([random_float(s) for _ in range(16)])
    kat["srand_seed"] = np.array(seeds, np.uint32)
    kat["rf_seq"] = np.array(seqs, np.float32)
    # transcendentals
    xb = np.concatenate([np.linspace(0, 2 * np.pi, 257)[:-1], rng.uniform(0, 6.2831853, 256)]).astype(np.float32)
    kat["sc_in"] = xb
    kat["sc_out"] = np.array([mc_sincos(x) for x in xb], np.float32)
    xl = np.concatenate([rng.uniform(1.2e-7, 1.0, 256), [1.0, 0.5, 2 ** -23, 0.70710677, 1.4142135, 3.0, 1e-30,
                                                          1e-40]]).astype(np.float32)
    kat["log_in"] = xl
    kat["log_out"] = np.array([mc_log(x) for x in xl], np.float32)
    xe = np.concatenate([rng.uniform(-140, 20, 256), [0.0, -0.5, 0.5, -126.5, -149.0, -10.25]]).astype(np.float32)
    kat["exp2_in"] = xe
    kat["exp2_out"] = np.array([mc_exp2(x) for x in xe], np.float32)
    px = np.concatenate([rng.uniform(0, 1, 128), [0.0, 1.0, 0.999]]).astype(np.float32)
    py = np.concatenate([rng.uniform(2, 100, 128), [50.0, 2.0, 100.0]]).astype(np.float32)
    kat["pow_in"] = np.stack([px, py], 1)
    kat["pow_out"] = np.array([mc_pow(a, b) for a, b in zip(px, py)], np.float32)
    # sampler
    rr_in, rr_seed, rr_rough, rr_out = [], [], [], []
    for k in range(128):
        d = rng.normal(size=3)
        d = (d / np.linalg.norm(d)).astype(np.float32)
        rough = f32([0.0, 0.01, 0.2, 0.5, 0.8, 1.0, rng.uniform()][k % 7])
        s = [int(v) for v in rng.integers(0, 2**32, 3, dtype=np.uint64)]
        rr_in.append(d)
        rr_seed.append(list(s))
        rr_rough.append(rough)
        rr_out.append(random_ray(list(s), d, rough))
    kat["rr_dir"] = np.array(rr_in, np.float32)
    kat["rr_seed"] = np.array(rr_seed, np.uint32)
    kat["rr_rough"] = np.array(rr_rough, np.float32)
    kat["rr_out"] = np.array(rr_out, np.float32)
    return kat


def make_prim_kat(rng, prims_by_scene):
    recs, O, D, shape, dist, dr, pl, pg = [], [], [], [], [], [], [], []
    for recs_scene in prims_by_scene:
        for rec in recs_scene:
            if int(rec[48]) not in (1, 2, 3, 5):
                continue
            c = rec[12:15].astype(np.float64)
            size = float(np.linalg.norm(rec[0:3])) + float(np.linalg.norm(rec[4:7])) + float(np.linalg.norm(rec[8:11]))
            for _ in range(6):
                o = (c + rng.normal(scale=300, size=3)).astype(np.float32)
                tgt = c + rng.normal(scale=0.25 * min(size, 300.0), size=3)
                d = (tgt - o)
                d = (d / np.linalg.norm(d)).astype(np.float32)
                b = intersect_prim(rec, list(o), list(d))
                recs.append(rec)
                O.append(o)
                D.append(d)
                shape.append(b["shape"])
                dist.append(b["dist"])
                dr.append(b["dir"])
                pl.append(b["pl"])
                pg.append(b["pg"])
    return {"ip_rec": np.array(recs, np.float32), "ip_O": np.array(O, np.float32), "ip_D": np.array(D, np.float32),
            "ip_shape": np.array(shape, np.int32), "ip_dist": np.array(dist, np.float32),
            "ip_dir": np.array(dr, np.int32), "ip_pl": np.array(pl, np.float32), "ip_pg": np.array(pg, np.float32)}


def cone_record(rng):
    """A PrimData record (scene.h:64-73) of a cone at a random pose: T·Rz·Ry·S in float32,
    inverse via float64."""
    ang = rng.uniform(-np.pi, np.pi, 2)
    cz, sz, cy, sy = np.cos(ang[0]), np.sin(ang[0]), np.cos(ang[1]), np.sin(ang[1])
    Rz = np.array([[cz, -sz, 0, 0], [sz, cz, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]])
    Ry = np.array([[cy, 0, sy, 0], [0, 1, 0, 0], [-sy, 0, cy, 0], [0, 0, 0, 1]])
    S = np.diag(list(rng.uniform(5, 40, 3)) + [1.0])
    T = np.eye(4)
    T[:3, 3] = rng.uniform(-100, 100, 3)
    M = (T @ Rz @ Ry @ S).astype(np.float32)
    inv = np.linalg.inv(M.astype(np.float64)).astype(np.float32)
    rec = np.zeros(64, np.float32)
    rec[0:16] = M.T.reshape(-1)          # column-major
    rec[16:32] = inv.T.reshape(-1)
    rec[32:48] = rec[0:16]
    rec[48] = 4.0
    rec[52:56] = [0.9, 0.9, 0.0, 1.0]
    rec[56:60] = [0.3, 0.6, 0.0, 0.0]
    return rec


def make_cone_kat(rng):
    recs, O, D, shape, dist, dr, pl, pg = [], [], [], [], [], [], [], []
    for _ in range(8):
        rec = cone_record(rng)
        c = rec[12:15].astype(np.float64)
        for _ in range(12):
            o = (c + rng.normal(scale=120, size=3)).astype(np.float32)
            d = (c + rng.normal(scale=15, size=3) - o)
            d = (d / np.linalg.norm(d)).astype(np.float32)
            b = intersect_prim(rec, list(o), list(d))
            recs.append(rec); O.append(o); D.append(d)
            shape.append(b["shape"]); dist.append(b["dist"]); dr.append(b["dir"]); pl.append(b["pl"]); pg.append(b["pg"])
    return {"cone_rec": np.array(recs, np.float32), "cone_O": np.array(O, np.float32),
            "cone_D": np.array(D, np.float32), "cone_shape": np.array(shape, np.int32),
            "cone_dist": np.array(dist, np.float32), "cone_dir": np.array(dr, np.int32),
            "cone_pl": np.array(pl, np.float32), "cone_pg": np.array(pg, np.float32)}


def make_sampler_kat(rng, k=24):
    """DrawSampling point clouds: tp/sampling_base.vert:23-26 seeding, tp/hsphere.vert main."""
    nrm, seeds, rough, nbu, out = [], [], [], [], []
    for case in range(6):
        n = rng.normal(size=3).astype(np.float32)
        fs = rng.uniform(0, 1, 3).astype(np.float32)
        r = np.float32([1.0, 0.5, 0.9, 0.0, 1.0, 0.25][case])
        nb = [3, 3, 2, 3, 5, 3][case]
        D = normalize([f32(v) for v in n])
        pts = []
        for v in range(k):
            step = (v * nb) & 0xFFFFFFFF
            base = [int(x) for x in fs.view(np.uint32)]
            seed = [(base[0] + step * 11) & 0xFFFFFFFF, (base[1] + step * 43) & 0xFFFFFFFF,
                    (base[2] + step * 67) & 0xFFFFFFFF]
            pts.append(random_ray(seed, D, r))
        nrm.append(n); seeds.append(fs); rough.append(r); nbu.append(nb); out.append(pts)
    return {"smp_normal": np.array(nrm, np.float32), "smp_fseed": np.array(seeds, np.float32),
            "smp_rough": np.array(rough, np.float32), "smp_nb": np.array(nbu, np.int32),
            "smp_out": np.array(out, np.float32)}


IMAGES = [  # (scene, variant, W, H, first_pass, spp, bounces, ior, light)
    (1, 0, 32, 24, 1, 4, 3, 1.0, 1.2), (2, 0, 32, 24, 1, 2, 8, 1.0, 1.2), (3, 0, 32, 24, 1, 2, 8, 1.0, 1.2),
    (4, 0, 32, 24, 1, 2, 8, 1.0, 1.2), (5, 0, 32, 24, 1, 2, 8, 1.0, 1.2), (6, 0, 32, 24, 1, 4, 8, 1.0, 1.2),
    (6, 0, 32, 24, 1, 4, 8, 1.5, 0.443), (7, 0, 32, 24, 1, 2, 8, 1.0, 1.2), (8, 0, 32, 24, 1, 2, 12, 1.0, 1.2),
    (1, 1, 32, 24, 1, 2, 3, 1.0, 1.2), (6, 2, 32, 24, 1, 2, 3, 1.0, 1.2), (6, 0, 16, 12, 20, 50, 4, 1.0, 1.2),
]


def image_name(c):
    s, v, W, H, p, n, B, ior, li = c
    return f"img_s{s}_v{v}_{W}x{H}_p{p}_n{n}_B{B}_ior{ior}_li{li}.npy"


def pure_refraction_scene():
    """A scene for the refraction branch no reference scene reaches (alpha < 1, shininess 0:
    montecarlo.frag:139-146): glass sphere and cylinder over a diffuse floor, a reflective
    cube, an emissive quad — built with the numpy restatement of the producer (scene.h add_* +
    finalize, scene_restate.py)."""
    def T(tx, ty, tz, sx, sy, sz):   # translate · scale, column-major
        m = np.eye(4, dtype=np.float32)
        m[0, 0], m[1, 1], m[2, 2] = sx, sy, sz
        m[0, 3], m[1, 3], m[2, 3] = tx, ty, tz
        return m.T.reshape(-1)
    ops = [(5, T(0, 0, 150, 40, 40, 1), [1.0, 1.0, 1.0, 1.0, 0.0, 0.0, 20.0]),
           (1, T(-40, 0, 0, 45, 45, 45), [0.7, 0.9, 0.8, 0.4, 0.0, 0.3, 0.0]),
           (3, T(70, 30, 0, 30, 30, 50), [0.9, 0.6, 0.6, 0.6, 0.0, 0.8, 0.0]),
           (2, T(0, 0, -60, 400, 400, 5), [0.8, 0.8, 0.8, 1.0, 0.0, 0.5, 0.0]),
           (2, T(30, -90, -20, 25, 25, 25), [0.5, 0.5, 0.9, 1.0, 0.6, 0.4, 0.0])]
    return scene_restate.custom([(t, np.asarray(m, np.float32), np.asarray(a, np.float32)) for t, m, a in ops])


PATH_CASES = [  # (scene id or 0 = pure_refraction_scene, light, ior, bounces, samples)
    (1, 1.2, 1.0, 3, 64), (6, 1.2, 1.0, 8, 64), (6, 0.443, 1.5, 8, 64), (8, 1.2, 1.0, 12, 64),
    (0, 1.2, 1.5, 8, 64),
]
# the other reference scenes (second RNG stream, appended after the cases above so those stay
# bit-identical): box of balls, Menger sponges, open box, material grid (IOR 1.5 too)
PATH_CASES_2 = [
    (2, 1.2, 1.0, 8, 48), (3, 1.2, 1.0, 8, 48), (4, 1.2, 1.0, 8, 48), (5, 1.2, 1.0, 8, 48),
    (5, 1.2, 1.5, 8, 32), (7, 1.2, 1.0, 8, 48),
]


# the two other tp/ programs (variant 1 = montecarlo_mat.frag, 2 = montecarlo_mat_tr.frag), third
# RNG stream, appended last: (scene, light, ior, bounces, samples, variant)
VARIANT_CASES = [(1, 1.2, 1.0, 8, 16, 1), (6, 1.2, 1.0, 8, 16, 1), (8, 1.2, 1.0, 12, 16, 1),
                 (1, 1.2, 1.0, 8, 16, 2), (6, 1.2, 1.0, 8, 16, 2), (8, 1.2, 1.0, 12, 16, 2)]


def make_path_kat(rng, cases=PATH_CASES, rng2=None, cases2=(), rng3=None, cases3=()):
    """Whole samples of the integrator (pixel, pass) at 1920×1080 with the numpy restatement
    above, on scene buffers and a camera from the numpy restatement of the host producer
    (scene_restate.py, round 5: no longer the oracle's): the oracle must reproduce every one bit
    for bit (tests/test_oracle_paths.py)."""
    W, H = 1920, 1080
    ipv, iv = scene_restate.camera(W, H)
    out = {k: [] for k in ("scene", "light", "ior", "bounces", "x", "y", "npass", "rgb", "trace", "variant")}
    custom = pure_refraction_scene()
    for scene_id, li, ior, B, n, variant, rng in ([c + (0, rng) for c in cases] + [c + (0, rng2) for c in cases2] +
                                                  [c + (rng3,) for c in cases3]):
        prims, nodes, leaves, depth, _ = custom if scene_id == 0 else scene_restate.build(scene_id, li)
        for k in range(n):
            # pixels near the image centre (objects) or anywhere; every 8th sample is drawn
            # until its path ends on an emissive primitive (at most 400 draws), so the
            # emissive end of montecarlo.frag:175-176 is covered
            for _ in range(400 if k % 8 == 7 else 1):
                if k % 2 == 0:
                    x, y = int(rng.integers(W // 4, 3 * W // 4)), int(rng.integers(H // 4, 3 * H // 4))
                else:
                    x, y = int(rng.integers(0, W)), int(rng.integers(0, H))
                npass = int(rng.integers(1, 84001)) if k % 3 else int(rng.integers(1, 33))
                rgb, tr = sample(prims, nodes, leaves, depth, ipv, iv, W, H, x, y, npass, B, ior, variant=variant)
                if tr[-1] == "E" or variant:
                    break
            for key, val in (("scene", scene_id), ("light", li), ("ior", ior), ("bounces", B), ("x", x), ("y", y),
                             ("npass", npass), ("rgb", rgb), ("trace", "".join(tr)), ("variant", variant)):
                out[key].append(val)
    kat = {"path_" + k: np.array(v) for k, v in out.items()}
    kat["path_rgb"] = np.array(out["rgb"], np.float32)
    kat["path_light"] = np.array(out["light"], np.float32)
    kat["path_ior"] = np.array(out["ior"], np.float32)
    kat["path_trace"] = np.array(out["trace"], "U32")
    kat["custom_prims"], kat["custom_nodes"], kat["custom_leaves"] = custom[0], custom[1].reshape(-1), custom[2]
    kat["custom_depth"] = np.array(custom[3], np.int32)
    kat["path_W"], kat["path_H"] = np.array(W, np.int32), np.array(H, np.int32)
    return kat


def main():
    from oracle import oracle as orc   # renders the img_*.npy regression images only
    if len(sys.argv) > 1 and sys.argv[1] == "paths":   # paths.npz only (round-2 addition)
        kat = make_path_kat(np.random.default_rng(20250216), PATH_CASES,
                            np.random.default_rng(20251016), PATH_CASES_2,
                            np.random.default_rng(20251017), VARIANT_CASES)
        np.savez_compressed(os.path.join(HERE, "paths.npz"), **kat)
        codes = "".join(kat["path_trace"].tolist())
        print("wrote paths.npz:", len(kat["path_x"]), "samples; branch counts",
              {c: codes.count(c) for c in "SERTMmFXIV"})
        return
    rng = np.random.default_rng(20241008)
    kat = make_kat(rng)
    prims = [scene_restate.build(s)[0] for s in (1, 2, 3, 6, 8)]
    prims = [p[: 24] for p in prims]
    kat.update(make_prim_kat(rng, prims))
    rng2 = np.random.default_rng(20241009)          # round-1 additions: cone + sampler
    kat.update(make_cone_kat(rng2))
    kat.update(make_sampler_kat(rng2))
    np.savez_compressed(os.path.join(HERE, "kat.npz"), **kat)
    for c in IMAGES:
        s, v, W, H, p, n, B, ior, li = c
        pr, nodes, leaves, d, _ = scene_restate.build(s, li)
        ipv, iv = scene_restate.camera(W, H)
        acc, _ = orc.render(pr, nodes, leaves, d, ipv, iv, W, H, p, n, 0.0, B, ior, v)
        np.save(os.path.join(HERE, image_name(c)), acc)
    print("wrote kat.npz and", len(IMAGES), "images")


if __name__ == "__main__":
    main()
