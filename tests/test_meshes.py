"""Triangle-mesh instances on CPU: the product's host producer vs the
oracle's independent restatement, the instance record, and the oracle's mesh traversal vs a
brute-force evaluation of every triangle."""
import numpy as np
import pytest

from mcpt import meshes


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


MESHES = {"cube": meshes.cube(), "sphere": meshes.uv_sphere(20, 10), "torus": meshes.torus(24, 12)}


def mesh_scene(mcpt_mod, flat=False):
    T, M = mcpt_mod.Transfo, mcpt_mod.material
    s = mcpt_mod.Scene()
    s.add_cube(T.mul(T.translate(0, 0, -51), T.scale(500, 500, 1)), M([0.9, 0.9, 0.9, 1], 0.3, 0.95))
    ids = {k: s.add_mesh(v, n, t, bb) for k, (v, n, t, bb) in MESHES.items()}
    s.place_mesh(ids["cube"], T.mul(T.translate(-80, 30, -10), T.rotateZ(30), T.scale(30, 30, 40)),
                 M([0.9, 0.1, 0.1, 1], 0.5, 0.8))
    s.place_mesh(ids["sphere"], T.mul(T.translate(60, -20, 0), T.scale(45)), M([0.1, 0.9, 0.9, 0.4], 0.7, 0.9))
    s.place_mesh(ids["torus"], T.mul(T.translate(0, 80, 10), T.rotateX(60), T.scale(50)),
                 M([0.9, 0.9, 0.1, 1], 0.0, 0.0))
    s.place_mesh(ids["torus"], T.mul(T.translate(-10, -90, -20), T.rotateY(-30), T.scale(35)),
                 M([0.2, 0.9, 0.2, 1], 0.8, 0.99))
    s.add_sphere(T.mul(T.translate(0, 0, 20), T.scale(20)), M([0.9, 0, 0.9, 0.2], 0.6, 0.7))
    s.add_oriented_quad(T.mul(T.translate(0, 0, 160), T.rotateX(180), T.scale(70, 70, 1)),
                        mcpt_mod.light([0.9, 0.9, 0.9, 1], 24))
    s.finalize()
    return s


@pytest.mark.parametrize("name", sorted(MESHES))
def test_mesh_bvh_matches_oracle(mcpt_mod, oracle_mod, name):
    v, n, t, bb = MESHES[name]
    s = mcpt_mod.Scene()
    mid = s.add_mesh(v, n, t, bb)
    s.place_mesh(mid, np.eye(4, dtype=np.float32), mcpt_mod.material([1, 1, 1, 1]))
    s.finalize()
    mb = s.mesh_buffers()
    d, nodes, leaves = oracle_mod.mesh_bvh(v, t)
    assert mb["info"].tolist() == [[0, 0, d, 0]]
    assert np.array_equal(bits(mb["nodes"]), bits(nodes))
    assert np.array_equal(mb["leaves"], leaves)
    assert sorted(leaves[leaves >= 0].tolist()) == list(range(len(t)))
    assert np.array_equal(mb["tris"], t.astype(np.int32))
    assert np.array_equal(bits(mb["verts"]), bits(v)) and np.array_equal(bits(mb["normals"]), bits(n))


def test_instance_record(mcpt_mod):
    """ScenePrimitives::add_mesh (scene.cpp:56-67): transfo = trf · BB.matrix(), inverse = trf^-1,
    mesh transfo = trf, type (0, mesh line), area 0."""
    T = mcpt_mod.Transfo
    s = mesh_scene(mcpt_mod)
    prims, _, _ = s.buffers()
    mesh_recs = prims[prims[:, 48] == 0]
    assert len(mesh_recs) == 4
    trf = T.mul(T.translate(60, -20, 0), T.scale(45))
    rec = [r for r in mesh_recs if np.array_equal(bits(r[32:48]), bits(trf))][0]
    bb = MESHES["sphere"][3]
    c = (bb[:3] + bb[3:]) / np.float32(2)
    sc = (bb[3:] - bb[:3]) / np.float32(2)
    assert np.array_equal(bits(rec[:16]), bits(T.mul(trf, T.mul(T.translate(*c), T.scale(*sc)))))
    assert rec[49] == 1.0 and rec[59] == 0.0          # mesh id (add order), area
    inv = np.linalg.inv(trf.reshape(4, 4).T.astype(np.float64)).astype(np.float32).T.reshape(-1)
    assert np.allclose(rec[16:32], inv, rtol=1e-6, atol=1e-7)


def test_mesh_buffers_layout(mcpt_mod):
    s = mesh_scene(mcpt_mod)
    mb = s.mesh_buffers()
    nv = [len(MESHES[k][0]) for k in ("cube", "sphere", "torus")]
    nt = [len(MESHES[k][2]) for k in ("cube", "sphere", "torus")]
    assert mb["info"][:, 3].tolist() == [0, nt[0], nt[0] + nt[1]]
    sph = mb["tris"][nt[0]:nt[0] + nt[1]]                            # global vertex ids
    assert sph.min() >= nv[0] and sph.max() < nv[0] + nv[1]
    assert mb["verts"].shape == (sum(nv), 3)


def _np_closest_triangle(v, t, O, D, Ol, trf):
    """Brute force over all triangles, the reference's float ops (numpy float32 + exact fma)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import gen_golden as g
    f32 = np.float32
    best = (f32(3.402823e38), -1)
    for k, tri in enumerate(t):
        A, B, C = ([f32(x) for x in v[i]] for i in tri)
        e1, e2 = g.vsub(B, A), g.vsub(C, A)
        h = g.cross(D, e2)
        det = g.dot3(e1, h)
        if abs(det) < f32(1e-10):
            continue
        inv = f32(f32(1.0) / det)
        sv = g.vsub(O, A)
        u = f32(g.dot3(sv, h) * inv)
        if u < 0 or u > 1:
            continue
        q = g.cross(sv, e1)
        w = f32(g.dot3(D, q) * inv)
        if w < 0 or f32(u + w) > 1:
            continue
        a = f32(g.dot3(e2, q) * inv)
        if a > f32(1e-10):
            Pg = g.xpoint(trf, g.vadd(O, g.vmul(D, a)))
            dist = g.length(g.vsub(Ol, Pg))
            if dist < best[0]:
                best = (dist, k)
    return best


def test_oracle_mesh_traversal_vs_brute_force(mcpt_mod, oracle_mod):
    """With a mesh-only scene, the oracle's closest hit (scene BVH → instance → mesh BVH) is
    the brute-force closest triangle, bit for bit (the boxes only cull)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import gen_golden as g
    T = mcpt_mod.Transfo
    v, n, t, bb = MESHES["torus"]
    s = mcpt_mod.Scene()
    mid = s.add_mesh(v, n, t, bb)
    trf = T.mul(T.translate(5, -3, 2), T.rotateX(40), T.scale(20))
    s.place_mesh(mid, trf, mcpt_mod.material([1, 1, 1, 1]))
    s.place_mesh(mid, T.mul(T.translate(500, 0, 0), T.scale(1)), mcpt_mod.material([1, 1, 1, 1]))
    s.finalize()
    prims, nodes, leaves = s.buffers()
    mv = oracle_mod.MeshView(s.mesh_buffers())
    rng = np.random.default_rng(4)
    o = rng.uniform(-60, 60, (60, 3)).astype(np.float32)
    tgt = rng.uniform(-15, 15, (60, 3)).astype(np.float32)
    d = (tgt - o).astype(np.float32)
    oi, of = oracle_mod.trace(prims, nodes, leaves, s.depth(), o, d, meshes=mv)
    k = [i for i in range(len(prims)) if np.array_equal(bits(prims[i][32:48]), bits(trf))][0]
    rec = prims[k]
    hits = 0
    for i in range(len(o)):
        Oi = g.xpoint(rec[16:32], list(o[i]))
        Di = g.normalize(g.xdir(rec[16:32], list(d[i])))
        dist, tri = _np_closest_triangle(v, t, Oi, Di, [np.float32(x) for x in o[i]], rec[32:48])
        if tri >= 0:
            hits += 1
            assert oi[i, 0] == 0 and oi[i, 1] == k and oi[i, 2] == tri, i
            assert bits(of[i, 0]) == bits(dist), i
        else:
            assert oi[i, 0] == -1, i
    assert hits > 15
