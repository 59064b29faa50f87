"""Fuzz: random scenes (tests/fuzz_scenes.py) rendered on the GPU vs the oracle, bit-exact,
over random image sizes, pass ranges, bounce budgets, refraction indices, shader variants
and kernel schedules (traversal mode, walk suspension, leaf batching); plus ray queries."""
import numpy as np
import pytest

from fuzz_scenes import build_product, random_ops

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def renderer(mcpt_mod):
    r = mcpt_mod.Renderer(0)
    yield r
    r.close()


@pytest.mark.parametrize("seed", range(96))
def test_random_scene_render(mcpt_mod, oracle_mod, renderer, seed):
    rng = np.random.default_rng(1000 + seed)
    ops = random_ops(mcpt_mod, seed)
    sc = build_product(mcpt_mod, ops)
    prims, nodes, leaves = sc.buffers()
    W, H = int(rng.integers(8, 49)), int(rng.integers(8, 41))
    first, S, B = int(rng.integers(1, 80)), int(rng.integers(1, 5)), int(rng.integers(0, 11))
    ior = 1.0 if rng.random() < 0.4 else float(rng.uniform(1.05, 2.0))
    variant = 0 if rng.random() < 0.8 else int(rng.integers(1, 3))
    traversal = int(rng.integers(1, 4))
    walk_exit = int(rng.choice([-1, 0, 4, 16, 40]))
    leaf_batch = int(rng.choice([-1, 0, 2, 8, 64]))
    renderer.set_traversal(traversal)
    renderer.set_walk_exit(walk_exit)
    renderer.set_leaf_batch(leaf_batch)
    try:
        renderer.upload_scene(sc)
        renderer.set_target(W, H)
        ipv, iv = mcpt_mod.camera_canonical(W, H)
        renderer.render(ipv, iv, first, S, 0.0, B, ior, variant)
        gpu, n = renderer.read_accum()
    finally:
        renderer.set_traversal(0)
        renderer.set_walk_exit(-1)
        renderer.set_leaf_batch(-1)
    ref, _ = oracle_mod.render(prims, nodes, leaves, sc.depth(), ipv, iv, W, H, first, S, 0.0, B, ior, variant)
    assert n == S
    bad = int((bits(gpu) != bits(ref.reshape(gpu.shape))).sum())
    assert bad == 0, (f"seed {seed}: {bad} channels differ (W {W} H {H} first {first} S {S} B {B} ior {ior} "
                      f"variant {variant} traversal {traversal} walk_exit {walk_exit} leaf_batch {leaf_batch})")


@pytest.mark.parametrize("seed", range(24))
def test_random_scene_queries(mcpt_mod, oracle_mod, renderer, seed):
    rng = np.random.default_rng(2000 + seed)
    sc = build_product(mcpt_mod, random_ops(mcpt_mod, 500 + seed))
    prims, nodes, leaves = sc.buffers()
    renderer.upload_scene(sc)
    o = rng.uniform(-200, 200, (3000, 3)).astype(np.float32)
    d = (rng.uniform(-60, 60, (3000, 3)) - o).astype(np.float32)
    for any_hit in (False, True):
        hits = renderer.trace(o, d, any_hit=any_hit)
        oi, of = oracle_mod.trace(prims, nodes, leaves, sc.depth(), o, d, any_hit=any_hit)
        assert np.array_equal(hits["shape"], oi[:, 0])
        hit = oi[:, 0] >= 0
        assert np.array_equal(hits["prim"][hit], oi[hit, 1]) and np.array_equal(hits["dir"][hit], oi[hit, 2])
        flat = np.concatenate([hits["dist"][:, None], hits["pl"], hits["pg"], hits["N"], hits["P"], hits["color"],
                               hits["material"]], axis=1)
        assert np.array_equal(bits(flat), bits(of))
