"""The stream schedule (MCPT_TRAVERSAL_STREAM): a pool of path slots, each
running (pixel, pass segment) units with their passes in order, advanced by iterations of a
trace kernel (persistent waves, lanes refilled from the ray queue) and a shade kernel.  Every
pool size and refill threshold must give the oracle's bits — pools far smaller than the launch
(many units per slot, long iteration tails), one-slot pools, partial sums over several segments,
launches split by the segment-sum budget."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STREAM = 3


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _render(mcpt_mod, r, sc, W, H, first, S, B, ior=1.0, slots=0, refill=-1, budget=None, variant=0):
    r.set_traversal(STREAM)
    r.set_stream_pool(slots, refill)
    if budget is not None:
        r.set_partial_budget(budget)
    try:
        r.upload_scene(sc)
        r.set_target(W, H)
        ipv, iv = mcpt_mod.camera_canonical(W, H)
        r.render(ipv, iv, first, S, 0.0, B, ior, variant)
        acc, n = r.read_accum()
        it = r.stream_iterations()
    finally:
        r.set_traversal(0)
        r.set_stream_pool(0, -1)
        r.set_partial_budget(1 << 30)
    assert n == S
    return acc, it


def _oracle(orc, sc, W, H, first, S, B, ior=1.0, variant=0):
    prims, nodes, leaves = sc.buffers()
    ipv, iv = orc.camera(W, H)
    acc, _ = orc.render(prims, nodes, leaves, sc.depth(), ipv, iv, W, H, first, S, 0.0, B, ior, variant)
    return acc


@pytest.fixture(scope="module")
def renderer(mcpt_mod):
    r = mcpt_mod.Renderer(0)
    yield r
    r.close()


@pytest.mark.parametrize("slots,refill", [(0, -1), (1, -1), (7, 0), (333, 17), (5000, 64), (100000, 56)])
@pytest.mark.parametrize("scene_id,B,ior", [(8, 12, 1.0), (3, 8, 1.0), (6, 8, 1.5), (5, 6, 1.3)])
def test_stream_pool_bit_exact(mcpt_mod, oracle_mod, renderer, scene_id, B, ior, slots, refill):
    """Passes 20..69 (three segments: partial sums and the combine kernel) at 40x24."""
    W, H, first, S = 40, 24, 20, 50
    if slots == 1:
        W, H, S = 8, 4, 40   # one slot runs every unit in turn: keep the launch small
    sc = mcpt_mod.Scene.reference(scene_id)
    gpu, it = _render(mcpt_mod, renderer, sc, W, H, first, S, B, ior, slots, refill)
    ref = _oracle(oracle_mod, sc, W, H, first, S, B, ior)
    assert it > 0
    bad = int((_bits(gpu) != _bits(ref.reshape(gpu.shape))).sum())
    assert bad == 0, f"{bad} channels differ (scene {scene_id} slots {slots} refill {refill})"


@pytest.mark.parametrize("first,S", [(1, 32), (5, 3), (33, 1)])
def test_stream_one_segment_adds_to_accumulator(mcpt_mod, oracle_mod, renderer, first, S):
    """One-segment launches add the unit sums straight into the accumulator; a second call adds
    on top (progressive), as the megakernel does."""
    W, H, B = 48, 32, 12
    sc = mcpt_mod.Scene.reference(8)
    renderer.set_traversal(STREAM)
    try:
        renderer.upload_scene(sc)
        renderer.set_target(W, H)
        ipv, iv = mcpt_mod.camera_canonical(W, H)
        renderer.render(ipv, iv, first, S, 0.0, B, 1.0, 0)
        renderer.render(ipv, iv, first + S, S, 0.0, B, 1.0, 0)
        gpu, n = renderer.read_accum()
    finally:
        renderer.set_traversal(0)
    prims, nodes, leaves = sc.buffers()
    oipv, oiv = oracle_mod.camera(W, H)
    acc, _ = oracle_mod.render(prims, nodes, leaves, sc.depth(), oipv, oiv, W, H, first, S, 0.0, B, 1.0, 0)
    ref, _ = oracle_mod.render(prims, nodes, leaves, sc.depth(), oipv, oiv, W, H, first + S, S, 0.0, B, 1.0, 0,
                               accum=acc)   # the same two calls
    assert n == 2 * S
    assert np.array_equal(_bits(gpu), _bits(ref.reshape(gpu.shape)))


def test_stream_budget_split_and_large_frame(mcpt_mod, oracle_mod, renderer):
    """A call cut into several launches by a one-segment budget, and a 1080p launch with a pool
    smaller than its units, against the per-lane megakernel bit for bit."""
    sc = mcpt_mod.Scene.reference(8)
    W, H, first, S, B = 64, 40, 7, 90, 12
    gpu, _ = _render(mcpt_mod, renderer, sc, W, H, first, S, B, budget=W * H * 12)
    ref = _oracle(oracle_mod, sc, W, H, first, S, B)
    assert np.array_equal(_bits(gpu), _bits(ref.reshape(gpu.shape)))
    W, H, first, S = 1920, 1080, 1, 64
    gpu, it = _render(mcpt_mod, renderer, sc, W, H, first, S, B, slots=1 << 20)
    lane = mcpt_mod.Renderer(0)
    try:
        lane.set_traversal(1)
        lane.upload_scene(sc)
        lane.set_target(W, H)
        ipv, iv = mcpt_mod.camera_canonical(W, H)
        lane.render(ipv, iv, first, S, 0.0, B, 1.0, 0)
        ref, _ = lane.read_accum()
    finally:
        lane.close()
    assert it > 0
    assert np.array_equal(_bits(gpu), _bits(ref))


def test_stream_falls_back_where_it_does_not_apply(mcpt_mod, oracle_mod, renderer):
    """Other tp/ programs and B = 0 run the per-lane walk under the stream setting (same bits)."""
    sc = mcpt_mod.Scene.reference(8)
    for variant, B in ((1, 3), (2, 3), (0, 0)):
        gpu, it = _render(mcpt_mod, renderer, sc, 24, 16, 1, 2, B, variant=variant)
        ref = _oracle(oracle_mod, sc, 24, 16, 1, 2, B, variant=variant)
        assert it == 0
        assert np.array_equal(_bits(gpu), _bits(ref.reshape(gpu.shape)))


@pytest.mark.parametrize("scene_id,B", [(8, 12), (3, 8)])
def test_stream_lds_nodes_variant(mcpt_mod, oracle_mod, renderer, monkeypatch, scene_id, B):
    """The trace kernel with the BVH nodes staged in LDS (MCPT_STREAM_LDS_NODES=1, off by
    default) gives the same bits."""
    monkeypatch.setenv("MCPT_STREAM_LDS_NODES", "1")
    sc = mcpt_mod.Scene.reference(scene_id)
    gpu, it = _render(mcpt_mod, renderer, sc, 40, 24, 20, 50, B, slots=300)
    ref = _oracle(oracle_mod, sc, 40, 24, 20, 50, B)
    assert it > 0
    assert np.array_equal(_bits(gpu), _bits(ref.reshape(gpu.shape)))
