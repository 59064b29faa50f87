"""Host scene producer (libmcpt C++, the product) vs the oracle's restatement, and BVH
invariants.  CPU only: these calls never touch a GPU."""
import numpy as np
import pytest

# SURVEY.md §8 per-scene table: prims, depth
SCENES = {1: (9, 4), 2: (14, 4), 3: (410, 9), 4: (13, 4), 5: (122, 7), 6: (6, 3), 7: (491, 9), 8: (895, 10)}


def bits(a):
    return np.asarray(a).view(np.uint32)


@pytest.mark.parametrize("sid", sorted(SCENES))
def test_reference_scene_buffers_match_oracle(mcpt_mod, oracle_mod, sid):
    s = mcpt_mod.Scene.reference(sid, 1.2)
    assert (s.nb_prim(), s.depth()) == SCENES[sid]
    p, n, l = s.buffers()
    op, on, ol, od, oe = oracle_mod.scene(sid, 1.2)
    assert od == s.depth() and oe == s.nb_emissives()
    assert np.array_equal(bits(p), bits(op))
    assert np.array_equal(bits(n), bits(on))
    assert np.array_equal(l, ol)


@pytest.mark.parametrize("sid", sorted(SCENES))
def test_bvh_invariants(mcpt_mod, sid):
    s = mcpt_mod.Scene.reference(sid)
    prims, nodes, leaves = s.buffers()
    n, d = s.nb_prim(), s.depth()
    assert nodes.shape == (2 ** (d + 1) - 1, 6) and leaves.shape == (2 ** d,)
    ids = leaves[leaves >= 0]
    assert sorted(ids.tolist()) == list(range(n))            # every prim in exactly one leaf
    # leaf pairs hold 1 or 2 prims; a lone prim sits in the left leaf with -1 on the right
    pairs = leaves.reshape(-1, 2)
    assert ((pairs[:, 0] >= 0)).all()
    # internal boxes are the merge of their children
    for i in range(2 ** d - 1):
        c1, c2 = nodes[2 * i + 1], nodes[2 * i + 2]
        assert np.array_equal(nodes[i][:3], np.minimum(c1[:3], c2[:3]))
        assert np.array_equal(nodes[i][3:], np.maximum(c1[3:], c2[3:]))
    # emissive prims first (sortEmissiveFirst)
    emis = prims[:, 58] > 0
    ne = s.nb_emissives()
    assert emis[:ne].all() and not emis[ne:].any()
    # every prim's world AABB contains its transformed unit-cube corners
    for i in range(n):
        leaf = int(np.where(leaves == i)[0][0]) + 2 ** d - 1
        lo, hi = nodes[leaf][:3], nodes[leaf][3:]
        T = prims[i][:16].reshape(4, 4).T
        z = 0.0 if prims[i][48] == 5 else 1.0
        for c in [(-1, -1, -z), (1, 1, z), (1, -1, z), (-1, 1, -z)]:
            w = T @ np.array([*c, 1.0])
            assert (w[:3] >= lo - 1e-2 * (1 + np.abs(lo))).all() and (w[:3] <= hi + 1e-2 * (1 + np.abs(hi))).all()


def test_inverse_transforms(mcpt_mod):
    prims, _, _ = mcpt_mod.Scene.reference(8).buffers()
    for rec in prims[::37]:
        T = rec[:16].reshape(4, 4).T.astype(np.float64)
        I = rec[16:32].reshape(4, 4).T.astype(np.float64)
        assert np.allclose(I @ T, np.eye(4), atol=1e-4)
        assert np.array_equal(I[3], [0, 0, 0, 1])            # affine (the kernel uses rows 0..2)


def test_median_split_order(mcpt_mod):
    """depth-1 rounds of nth_element splits, axis x -> y -> z (bvh.cpp:34-60)."""
    s = mcpt_mod.Scene.reference(5)       # 122 spheres on a grid + ground
    prims, nodes, leaves = s.buffers()
    d = s.depth()
    # the root's two children split the prims at the median of the box centres along x
    left = [i for i in leaves[: 2 ** (d - 1)] if i >= 0]
    right = [i for i in leaves[2 ** (d - 1):] if i >= 0]
    assert abs(len(left) - len(right)) <= 1
    def cx(i):
        lo = nodes[np.where(leaves == i)[0][0] + 2 ** d - 1]
        return (lo[0] + lo[3]) / 2
    assert max(cx(i) for i in left) <= min(cx(i) for i in right)


def test_custom_scene_api(mcpt_mod, oracle_mod):
    """BVH_GPU_Scene add_* / finalize through the C ABI reproduces a reference builder."""
    import mcpt
    ref = mcpt.Scene.reference(6)
    rp, rn, rl = ref.buffers()
    s = mcpt.Scene()
    # rebuild scene 6 in montecarlo.cpp:756-770 order (ground, 4 spheres, light); after
    # sortEmissiveFirst the light (added last) was swapped with the ground into slot 0
    order = [5, 1, 2, 3, 4, 0]
    add = {1: s.add_sphere, 2: s.add_cube, 3: s.add_cylinder, 4: s.add_cone, 5: s.add_oriented_quad}
    for i in order:
        rec = rp[i]
        add[int(rec[48])](rec[:16], np.concatenate([rec[52:56], rec[56:59]]))
    s.finalize()
    p, n, l = s.buffers()
    assert np.array_equal(bits(p), bits(rp)) and np.array_equal(bits(n), bits(rn)) and np.array_equal(l, rl)


def test_set_material_and_errors(mcpt_mod):
    import mcpt
    s = mcpt.Scene.reference(6)
    prims, _, _ = s.buffers()
    m = np.concatenate([prims[3][52:56], [prims[3][56], 0.25, 0.0]]).astype(np.float32)
    s.set_material(3, m)
    assert s.buffers()[0][3][57] == np.float32(0.25)
    with pytest.raises(mcpt.MCPTError):
        s.set_material(3, np.array([1, 1, 1, 1, 0, 0, 5.0], np.float32))   # would break emissive-first order
    with pytest.raises(mcpt.MCPTError):
        mcpt.Scene.reference(9)
    e = mcpt.Scene()
    with pytest.raises(mcpt.MCPTError):
        e.finalize()                                                        # empty scene


def test_camera_matches_oracle_and_geometry(mcpt_mod, oracle_mod):
    for W, H in [(256, 256), (1920, 1080), (3840, 2160), (1280, 1000), (300, 900)]:
        a, b = mcpt_mod.camera_canonical(W, H)
        c, d = oracle_mod.camera(W, H)
        assert np.array_equal(bits(a), bits(c)) and np.array_equal(bits(b), bits(d))
    a, b = mcpt_mod.camera_canonical(1920, 1080)
    eye = b.reshape(4, 4).T @ np.array([0, 0, 0, 1.0])
    assert np.allclose(eye[:3], [0, -347.39, 61.25], atol=0.05)


# the numpy restatement of the host producer written from the reference's C++ text
# (tests/golden/scene_restate.py; round 5): the source of tests/golden/paths.npz' scene buffers
# and cameras.  Product, oracle and restatement: three producers, bit for bit.
@pytest.mark.parametrize("sid", sorted(SCENES))
def test_reference_scene_buffers_match_numpy_restatement(mcpt_mod, oracle_mod, sid):
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import scene_restate as R
    for li in (1.2, 0.443):
        p, n, l, d, e = R.build(sid, li)
        s = mcpt_mod.Scene.reference(sid, li)
        sp, sn, sl = s.buffers()
        assert (d, e) == (s.depth(), s.nb_emissives())
        assert np.array_equal(bits(p), bits(sp)) and np.array_equal(bits(n), bits(sn)) and np.array_equal(l, sl)
        op, on, ol, od, oe = oracle_mod.scene(sid, li)
        assert (d, e) == (od, oe)
        assert np.array_equal(bits(p), bits(op)) and np.array_equal(bits(n), bits(on)) and np.array_equal(l, ol)


def test_camera_matches_numpy_restatement(mcpt_mod, oracle_mod):
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import scene_restate as R
    for W, H in ((1920, 1080), (3840, 2160), (256, 256), (32, 24), (1000, 1280), (64, 40)):
        a, b = R.camera(W, H)
        pa, pb = mcpt_mod.camera_canonical(W, H)
        oa, ob = oracle_mod.camera(W, H)
        assert np.array_equal(bits(a), bits(pa)) and np.array_equal(bits(b), bits(pb)), (W, H)
        assert np.array_equal(bits(a), bits(oa)) and np.array_equal(bits(b), bits(ob)), (W, H)


def test_nth_element_restatement_matches_libstdcxx(oracle_mod):
    """The restated std::nth_element (libstdc++ introselect, incl. the heap-select fallback)
    against the C++ library's own on adversarial and random inputs, through the oracle's
    mesh BVH builder (the same BVH_KDtree code path, with its nth_element calls)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import scene_restate as R
    rng = np.random.default_rng(5)
    for n in (2, 3, 4, 5, 7, 16, 33, 100, 257, 1000):
        for kind in ("random", "sorted", "reversed", "equal", "organ"):
            if kind == "random":
                keys = rng.integers(0, 50, n).astype(np.float32)
            elif kind == "sorted":
                keys = np.arange(n, dtype=np.float32)
            elif kind == "reversed":
                keys = np.arange(n, dtype=np.float32)[::-1].copy()
            elif kind == "equal":
                keys = np.zeros(n, np.float32)
            else:
                keys = np.concatenate([np.arange(n // 2), np.arange(n - n // 2)[::-1]]).astype(np.float32)
            for nth in sorted({0, n // 2, n - 1}):
                v = list(range(n))
                R.nth_element(v, 0, nth, n, lambda a, b: keys[a] < keys[b])
                ref = sorted(keys)
                assert keys[v[nth]] == ref[nth]
                assert all(keys[v[i]] <= keys[v[nth]] for i in range(nth)) and \
                    all(keys[v[i]] >= keys[v[nth]] for i in range(nth + 1, n))
    # exact element placement against libstdc++: the oracle's mesh BVH (BVH_KDtree over the
    # triangles' centres) and the restatement's kd_tree on the same centres and boxes
    v = rng.uniform(-1, 1, (300, 3)).astype(np.float32)
    t = rng.integers(0, 300, (701, 3)).astype(np.int32)
    depth, nodes, leaves = oracle_mod.mesh_bvh(v, t)
    cen, bbs = [], []
    for tri in t:
        p = v[tri]
        lo, hi = p.min(0), p.max(0)
        cen.append(np.array([np.float32(np.float32(lo[k] + hi[k]) / np.float32(2.0)) for k in range(3)], np.float32))
        bbs.append(np.concatenate([lo, hi]))
    d2, n2, l2 = R.kd_tree(cen, bbs)
    assert d2 == depth and np.array_equal(l2, leaves)
