"""Procedural triangle meshes for mesh instances.

The reference loads meshes with assimp or builds them procedurally (easycppogl/mesh.cpp);
these generators give the same kind of input — positions, per-vertex normals, triangle
index triplets and the Mesh::BB() box — as float32 / uint32 numpy arrays:

* cube(): Mesh::Cube (easycppogl/mesh.cpp:252-283): 24 vertices (4 per face, face normals),
  12 triangles, BB = [-1, 1]^3;
* uv_sphere(n_lon, n_lat): unit sphere, normals = positions, BB = [-1, 1]^3;
* torus(n_major, n_minor, r): ring radius 1, tube radius r, BB = [-1-r, 1+r]² × [-r, r].

Sizes grow quadratically with the tessellation, which is how mesh scenes reach HBM scale.
"""
from __future__ import annotations

import numpy as np

__all__ = ["cube", "uv_sphere", "torus"]


def cube():
    v, V = -1.0, 1.0
    pos = [(v, v, v), (V, v, v), (V, V, v), (v, V, v), (v, v, V), (V, v, V), (V, V, V), (v, V, V),
           (v, v, V), (v, v, v), (v, V, v), (v, V, V), (V, v, V), (V, v, v), (V, V, v), (V, V, V),
           (v, v, V), (V, v, V), (V, v, v), (v, v, v), (v, V, V), (V, V, V), (V, V, v), (v, V, v)]
    nrm = [(0, 0, -1)] * 4 + [(0, 0, 1)] * 4 + [(-1, 0, 0)] * 4 + [(1, 0, 0)] * 4 + [(0, -1, 0)] * 4 + \
          [(0, 1, 0)] * 4
    tri = [0, 3, 2, 0, 2, 1, 4, 5, 6, 4, 6, 7, 8, 11, 10, 8, 10, 9, 12, 13, 14, 12, 14, 15, 16, 19, 18, 16, 18,
           17, 20, 21, 22, 20, 22, 23]
    return (np.array(pos, np.float32), np.array(nrm, np.float32), np.array(tri, np.uint32).reshape(-1, 3),
            np.array([-1, -1, -1, 1, 1, 1], np.float32))


def uv_sphere(n_lon: int = 24, n_lat: int = 12):
    th = np.linspace(0.0, np.pi, n_lat + 1)
    ph = np.linspace(0.0, 2.0 * np.pi, n_lon + 1)
    T, Pp = np.meshgrid(th, ph, indexing="ij")
    pos = np.stack([np.sin(T) * np.cos(Pp), np.sin(T) * np.sin(Pp), np.cos(T)], -1).reshape(-1, 3)
    tris = []
    w = n_lon + 1
    for i in range(n_lat):
        for j in range(n_lon):
            a, b, c, d = i * w + j, i * w + j + 1, (i + 1) * w + j, (i + 1) * w + j + 1
            if i > 0:
                tris.append((a, c, b))
            if i < n_lat - 1:
                tris.append((b, c, d))
    pos = pos.astype(np.float32)
    return pos, pos.copy(), np.array(tris, np.uint32), np.array([-1, -1, -1, 1, 1, 1], np.float32)


def torus(n_major: int = 32, n_minor: int = 16, r: float = 0.35):
    u = np.linspace(0.0, 2.0 * np.pi, n_major + 1)
    v = np.linspace(0.0, 2.0 * np.pi, n_minor + 1)
    U, Vv = np.meshgrid(u, v, indexing="ij")
    ring = np.stack([np.cos(U), np.sin(U), np.zeros_like(U)], -1)
    nrm = np.stack([np.cos(Vv) * np.cos(U), np.cos(Vv) * np.sin(U), np.sin(Vv)], -1)
    pos = ring + r * nrm
    w = n_minor + 1
    tris = []
    for i in range(n_major):
        for j in range(n_minor):
            a, b, c, d = i * w + j, i * w + j + 1, (i + 1) * w + j, (i + 1) * w + j + 1
            tris.append((a, c, b))
            tris.append((b, c, d))
    bb = np.array([-1 - r, -1 - r, -r, 1 + r, 1 + r, r], np.float32)
    return (pos.reshape(-1, 3).astype(np.float32), nrm.reshape(-1, 3).astype(np.float32),
            np.array(tris, np.uint32), bb)
