"""GPU ray queries, the DrawSampling point cloud and a cone scene vs the oracle (bit-exact).

Covers SURVEY §8f rows 3-4: Cone_intersect / cone_inter_geom_info in a rendered scene, the
any-hit traversal (just_hit_bvh, hit_one_prim) and closest-hit queries (traverse_all_bvh,
intersect_one_prim) + intersection_info / colour / material, and the sampler visualiser.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def renderer(mcpt_mod):
    r = mcpt_mod.Renderer(0)
    yield r
    r.close()


def _rays(rng, n, spread=260.0):
    o = rng.uniform(-spread, spread, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    return o, d


def _check(hits, oi, of):
    assert np.array_equal(hits["shape"], oi[:, 0])
    hit = oi[:, 0] >= 0
    assert np.array_equal(hits["prim"][hit], oi[hit, 1])
    assert np.array_equal(hits["dir"][hit], oi[hit, 2])
    flat = np.concatenate([hits["dist"][:, None], hits["pl"], hits["pg"], hits["N"], hits["P"], hits["color"],
                           hits["material"]], axis=1)
    assert np.array_equal(bits(flat), bits(of))


@pytest.mark.parametrize("scene_id", [1, 2, 3, 4, 5, 6, 7, 8])
def test_trace_closest_and_any(mcpt_mod, oracle_mod, renderer, scene_id):
    sc = mcpt_mod.Scene.reference(scene_id)
    renderer.upload_scene(sc)
    prims, nodes, leaves = sc.buffers()
    o, d = _rays(np.random.default_rng(scene_id), 3000)
    for any_hit in (False, True):
        hits = renderer.trace(o, d, any_hit=any_hit)
        oi, of = oracle_mod.trace(prims, nodes, leaves, sc.depth(), o, d, any_hit=any_hit)
        _check(hits, oi, of)
    assert (hits["shape"] >= 0).sum() > 100


def test_trace_one_prim(mcpt_mod, oracle_mod, renderer):
    sc = mcpt_mod.Scene.reference(6)
    renderer.upload_scene(sc)
    prims, nodes, leaves = sc.buffers()
    o, d = _rays(np.random.default_rng(11), 2000)
    for k in range(sc.nb_prim()):
        for any_hit in (False, True):
            hits = renderer.trace(o, d, any_hit=any_hit, prim=k)
            oi, of = oracle_mod.trace(prims, nodes, leaves, sc.depth(), o, d, any_hit=any_hit, prim=k)
            _check(hits, oi, of)


def test_sampler_point_cloud(mcpt_mod, oracle_mod, renderer):
    rng = np.random.default_rng(2)
    for rough, nb in ((1.0, 3), (0.3, 2), (0.0, 3)):
        nrm = rng.normal(size=3).astype(np.float32)
        fs = rng.uniform(0, 1, 3).astype(np.float32)
        got = renderer.sample_hemisphere(nrm, fs, 20000, rough, nb)
        want = oracle_mod.sample_hemisphere(nrm, fs, 20000, rough, nb)
        assert np.array_equal(bits(got), bits(want))


def cone_scene(mcpt_mod, light=1.2):
    """A test scene (not one of the reference's 8): cones, cylinders, spheres, cubes and a
    quad light, built through the BVH_GPU_Scene-compatible API."""
    T, M = mcpt_mod.Transfo, mcpt_mod.material
    s = mcpt_mod.Scene()
    s.add_cube(T.mul(T.translate(0, 0, -51), T.scale(400, 400, 1)), M([0.9, 0.9, 0.9, 1], 0.3, 0.95))
    for k in range(5):
        a = 72.0 * k
        pose = T.mul(T.rotateZ(a), T.translate(90, 0, -10), T.rotateX(15.0 * k), T.scale(22, 22, 40))
        s.add_cone(pose, M([0.9, 0.2 * k, 0.1, 1.0 if k % 2 else 0.2], 0.5, 0.8))
    s.add_cylinder(T.mul(T.translate(0, 0, -20), T.scale(25, 25, 30)), M([0.1, 0.8, 0.9, 1], 0.7, 0.9))
    s.add_sphere(T.mul(T.translate(-40, 60, 20), T.scale(18)), M([0.9, 0.0, 0.9, 0.3], 0.6, 0.7))
    s.add_oriented_quad(T.mul(T.translate(0, 0, 150), T.rotateX(180), T.scale(60, 60, 1)),
                        mcpt_mod.light([0.9, 0.9, 0.9, 1], 20 * light))
    s.finalize()
    return s


@pytest.mark.parametrize("traversal", [1, 2, 3])
def test_cone_scene_render(mcpt_mod, oracle_mod, renderer, traversal):
    sc = cone_scene(mcpt_mod)
    prims, nodes, leaves = sc.buffers()
    assert (prims[:, 48] == 4).sum() == 5
    W, H, S, B = 64, 48, 3, 8
    renderer.set_traversal(traversal)
    renderer.upload_scene(sc)
    renderer.set_target(W, H)
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    renderer.render(ipv, iv, 1, S, 0.0, B, 1.3, 0)
    gpu, n = renderer.read_accum()
    renderer.set_traversal(0)
    ref, _ = oracle_mod.render(prims, nodes, leaves, sc.depth(), ipv, iv, W, H, 1, S, 0.0, B, 1.3, 0)
    assert n == S and np.isfinite(gpu).all()
    assert np.array_equal(bits(gpu), bits(ref))
    # the cones are actually seen: closest-hit queries along the camera's corner-to-centre rays
    o = np.tile(np.array([0.0, -347.39, 61.25], np.float32), (400, 1))
    tgt = np.random.default_rng(0).uniform([-120, -120, -40], [120, 120, 40], (400, 3)).astype(np.float32)
    hits = renderer.trace(o, tgt - o)
    assert (hits["shape"] == 4).sum() > 10
