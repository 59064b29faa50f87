"""Triangle-mesh instances on the GPU vs the oracle, bit-exact: renders
(both BVH walks, smooth and flat normals), ray queries, and the event counters."""
import numpy as np
import pytest

from test_meshes import mesh_scene

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def renderer(mcpt_mod):
    r = mcpt_mod.Renderer(0)
    yield r
    r.close()


@pytest.mark.parametrize("flat,walk_exit", [(False, -1), (True, -1), (False, 12), (False, 0), (False, 63)])
@pytest.mark.parametrize("traversal", [1, 2, 3])
def test_mesh_scene_render(mcpt_mod, oracle_mod, renderer, traversal, flat, walk_exit):
    sc = mesh_scene(mcpt_mod)
    prims, nodes, leaves = sc.buffers()
    W, H, S, B = 64, 48, 3, 8
    renderer.set_traversal(traversal)
    renderer.set_walk_exit(walk_exit)
    renderer.set_leaf_batch(4 if walk_exit == 0 else -1)
    renderer.set_flat_face(flat)
    renderer.upload_scene(sc)
    renderer.set_target(W, H)
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    renderer.render(ipv, iv, 1, S, 0.0, B, 1.2, 0)
    gpu, n = renderer.read_accum()
    renderer.set_traversal(0)
    renderer.set_walk_exit(-1)
    renderer.set_leaf_batch(-1)
    renderer.set_flat_face(False)
    mv = oracle_mod.MeshView(sc.mesh_buffers(), flat_face=flat)
    ref, _ = oracle_mod.render(prims, nodes, leaves, sc.depth(), ipv, iv, W, H, 1, S, 0.0, B, 1.2, 0, meshes=mv)
    assert n == S and np.isfinite(gpu).all()
    assert np.array_equal(bits(gpu), bits(ref))


def test_mesh_queries(mcpt_mod, oracle_mod, renderer):
    sc = mesh_scene(mcpt_mod)
    prims, nodes, leaves = sc.buffers()
    renderer.upload_scene(sc)
    mv = oracle_mod.MeshView(sc.mesh_buffers())
    rng = np.random.default_rng(9)
    o = rng.uniform(-200, 200, (4000, 3)).astype(np.float32)
    d = (rng.uniform(-80, 80, (4000, 3)) - o).astype(np.float32)
    for any_hit in (False, True):
        hits = renderer.trace(o, d, any_hit=any_hit)
        oi, of = oracle_mod.trace(prims, nodes, leaves, sc.depth(), o, d, any_hit=any_hit, meshes=mv)
        assert np.array_equal(hits["shape"], oi[:, 0])
        hit = oi[:, 0] >= 0
        assert np.array_equal(hits["prim"][hit], oi[hit, 1]) and np.array_equal(hits["dir"][hit], oi[hit, 2])
        flat = np.concatenate([hits["dist"][:, None], hits["pl"], hits["pg"], hits["N"], hits["P"], hits["color"],
                               hits["material"]], axis=1)
        assert np.array_equal(bits(flat), bits(of))
    assert (hits["shape"] == 0).sum() > 200          # mesh hits


def test_mesh_event_counters(mcpt_mod, oracle_mod, renderer):
    sc = mesh_scene(mcpt_mod)
    prims, nodes, leaves = sc.buffers()
    W, H, S = 40, 30, 2
    renderer.upload_scene(sc)
    renderer.set_target(W, H)
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    ev = renderer.render_counted(ipv, iv, 1, S, 0.0, 8, 1.0, 0)
    mv = oracle_mod.MeshView(sc.mesh_buffers())
    _, ref_ev = oracle_mod.render(prims, nodes, leaves, sc.depth(), ipv, iv, W, H, 1, S, 0.0, 8, 1.0, 0, meshes=mv)
    assert np.array_equal(ev, ref_ev), (ev, ref_ev)
    assert ev[9] > 0 and ev[10] > 0                   # triangle tests, mesh hit infos


def test_mesh_instances_require_meshes(mcpt_mod, renderer):
    sc = mesh_scene(mcpt_mod)
    prims, nodes, leaves = sc.buffers()
    renderer.upload_scene(prims=prims, nodes=nodes, leaves=leaves, depth=sc.depth(), nb_emissives=1)
    renderer.set_target(8, 8)
    ipv, iv = mcpt_mod.camera_canonical(8, 8)
    with pytest.raises(mcpt_mod.MCPTError):
        renderer.render(ipv, iv, 1, 1, 0.0, 3, 1.0, 0)
