"""BASELINE.json configurations at their full sizes: oracle checks on row subsets
(the oracle renders only the sampled rows) and size-independent properties over whole frames —
determinism, launch-split invariance at chunk boundaries, row-band shard invariance."""
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


def render(mcpt_mod, r, sc, W, H, first, S, B, ior=1.0, band_rows=8, world=1, rank=0, split=None):
    r.upload_scene(sc)
    r.set_target(W, H, band_rows, world, rank)
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    p = first
    for n in (split or [S]):
        r.render(ipv, iv, p, n, 0.0, B, ior, 0)
        p += n
    acc, n = r.read_accum()
    assert n == S
    return acc


def oracle_rows(oracle_mod, sc, W, H, first, S, B, rows, ior=1.0):
    """Oracle image restricted to `rows` (absolute frame rows)."""
    prims, nodes, leaves = sc.buffers()
    ipv, iv = oracle_mod.camera(W, H)
    out = {}
    for y in rows:
        ref, _ = oracle_mod.render(prims, nodes, leaves, sc.depth(), ipv, iv, W, H, first, S, 0.0, B, ior, 0,
                                   row_step=H, row_offset=int(y))
        out[int(y)] = ref[int(y)]
    return out


def test_c5_4k_shard_rows(mcpt_mod, oracle_mod, renderer):
    """C5 geometry: 3840x2160, 8-GPU row bands (rank 3), late passes of the 84,000-spp run."""
    sc = mcpt_mod.Scene.reference(6)
    W, H, first, S, B = 3840, 2160, 83_969, 2, 8
    part = render(mcpt_mod, renderer, sc, W, H, first, S, B, world=8, rank=3)
    rows = renderer.local_row_ids()
    pick = np.arange(5, len(rows), 67)
    ref = oracle_rows(oracle_mod, sc, W, H, first, S, B, rows[pick])
    for i in pick:
        assert np.array_equal(bits(part[i]), bits(ref[int(rows[i])])), f"4K row {rows[i]}"


def test_c4_scene8_rows(mcpt_mod, oracle_mod, renderer):
    """C4 workload: scene 8 (largest BVH), 1080p, B 12 (deep-BVH walk kernel)."""
    sc = mcpt_mod.Scene.reference(8)
    W, H, S, B = 1920, 1080, 2, 12
    img = render(mcpt_mod, renderer, sc, W, H, 1, S, B)
    rows = np.arange(11, H, 157)
    ref = oracle_rows(oracle_mod, sc, W, H, 1, S, B, rows)
    for y in rows:
        assert np.array_equal(bits(img[y]), bits(ref[int(y)])), f"scene 8 row {y}"


def test_c3_ior_roughness_rows(mcpt_mod, oracle_mod, renderer):
    """C3 workload: scene 6, IOR 1.5, roughness 0.5 on every non-emissive primitive."""
    sc = mcpt_mod.Scene.reference(6)
    prims, _, _ = sc.buffers()
    for i in range(sc.nb_prim()):
        rec = prims[i]
        if rec[58] <= 0:
            sc.set_material(i, np.concatenate([rec[52:56], [rec[56], 0.5, rec[58]]]).astype(np.float32))
    W, H, S, B = 1920, 1080, 2, 8
    img = render(mcpt_mod, renderer, sc, W, H, 1, S, B, ior=1.5)
    rows = np.arange(3, H, 119)
    ref = oracle_rows(oracle_mod, sc, W, H, 1, S, B, rows, ior=1.5)
    for y in rows:
        assert np.array_equal(bits(img[y]), bits(ref[int(y)])), f"C3 row {y}"


def test_c2_determinism_and_chunk_split(mcpt_mod, renderer):
    """C2 at full size: the same 64 passes twice, and split at the 32-pass chunk boundary."""
    sc = mcpt_mod.Scene.reference(6)
    a = render(mcpt_mod, renderer, sc, 1920, 1080, 1, 64, 8)
    b = render(mcpt_mod, renderer, sc, 1920, 1080, 1, 64, 8)
    c = render(mcpt_mod, renderer, sc, 1920, 1080, 1, 64, 8, split=[32, 32])
    assert np.array_equal(bits(a), bits(b))
    assert np.array_equal(bits(a), bits(c))
    assert np.isfinite(a).all() and (a >= 0).all() and a.mean() > 0


def test_c2_shards_cover_frame(mcpt_mod, renderer):
    """8 row-band shards of the 1080p frame are exactly the single-GPU frame's rows."""
    sc = mcpt_mod.Scene.reference(6)
    full = render(mcpt_mod, renderer, sc, 1920, 1080, 1, 4, 8)
    seen = np.zeros(1080, bool)
    for rank in range(8):
        part = render(mcpt_mod, renderer, sc, 1920, 1080, 1, 4, 8, world=8, rank=rank)
        rows = renderer.local_row_ids()
        assert not seen[rows].any()
        seen[rows] = True
        assert np.array_equal(bits(part), bits(full[rows]))
    assert seen.all()


@pytest.fixture(scope="module")
def big_mesh(mcpt_mod):
    from mcpt import meshes
    return meshes.big_mesh_scene(1_000_000)[0]


@pytest.mark.parametrize("traversal", [0, 1, 3])
def test_mesh_1m_rows(mcpt_mod, oracle_mod, renderer, big_mesh, traversal):
    """The HBM-sized mesh workload (bench.py --config mesh: two instances of a 1 M-triangle UV
    sphere, mesh BVH depth 20), 1080p, B 8, against the oracle's own mesh DFS on a row subset."""
    sc = big_mesh
    W, H, S, B = 1920, 1080, 2, 8
    renderer.set_traversal(traversal)
    try:
        img = render(mcpt_mod, renderer, sc, W, H, 1, S, B)
    finally:
        renderer.set_traversal(0)
    rows = np.arange(7, H, 149)
    prims, nodes, leaves = sc.buffers()
    ipv, iv = oracle_mod.camera(W, H)
    mv = oracle_mod.MeshView(sc.mesh_buffers())
    for y in rows:
        ref, _ = oracle_mod.render(prims, nodes, leaves, sc.depth(), ipv, iv, W, H, 1, S, 0.0, B, 1.0, 0,
                                   row_step=H, row_offset=int(y), meshes=mv)
        assert np.array_equal(bits(img[y]), bits(ref[int(y)])), f"1 M-triangle mesh scene row {y}"
    assert np.isfinite(img).all()


def test_mesh_split_items_same_bits(mcpt_mod, renderer, big_mesh, monkeypatch):
    """Work-item order + split items on the 1 M-triangle mesh workload (mcpt_order.hip): after
    the first launch the costliest items run first and the costliest of those in 4 pass
    ranges (the later pieces' per-pass values added by the combine after piece 0's sum).  Three
    64-pass calls equal the same passes in launch order without splits, bit for bit; debug slot
    63 shows that items were split."""
    W, H, B = 1920, 1080, 8
    renderer.set_traversal(1)
    try:
        monkeypatch.setenv("MCPT_ITEM_ORDER", "1")
        a = render(mcpt_mod, renderer, big_mesh, W, H, 1, 192, B, split=[64, 64, 64])
        n_split = int(renderer.debug_counters()[63])
        monkeypatch.setenv("MCPT_ITEM_ORDER", "0")
        b = render(mcpt_mod, renderer, big_mesh, W, H, 1, 192, B, split=[64, 64, 64])
    finally:
        renderer.set_traversal(0)
    assert n_split > 0
    assert np.array_equal(bits(a), bits(b))


def test_mesh_pass_stealing_same_bits(mcpt_mod, renderer, big_mesh, monkeypatch):
    """Pass stealing on the 1 M-triangle mesh workload (RenderParams::steal_vals): a lane whose
    pixel's passes are done renders the next unstarted pass of another pixel of its workgroup,
    every pass's value is stored and combine_steal_kernel sums each segment's passes from 0 in pass
    order.  Three 64-pass calls equal the same calls with MCPT_STEAL=0 bit for bit; debug slot 62
    counts the passes rendered for another lane's pixel."""
    W, H, B = 1920, 1080, 8
    renderer.set_traversal(1)
    try:
        monkeypatch.setenv("MCPT_STEAL", "1")
        renderer.debug_counters(reset=True)
        a = render(mcpt_mod, renderer, big_mesh, W, H, 1, 192, B, split=[64, 64, 64])
        n_stolen = int(renderer.debug_counters()[62])
        monkeypatch.setenv("MCPT_STEAL", "0")
        b = render(mcpt_mod, renderer, big_mesh, W, H, 1, 192, B, split=[64, 64, 64])
    finally:
        renderer.set_traversal(0)
    assert n_stolen > 0
    assert np.array_equal(bits(a), bits(b))


@pytest.fixture(scope="module")
def big_mesh4(mcpt_mod):
    from mcpt import meshes
    return meshes.big_mesh4_scene(1_000_000)[0]


@pytest.mark.parametrize("traversal", [0, 1])
def test_mesh_big_rows(mcpt_mod, oracle_mod, renderer, big_mesh4, traversal):
    """The mesh workload past the Infinity Cache (bench.py --config mesh_big: four distinct meshes
    of ~1 M triangles, one instance each, mesh BVHs of depth 20), 1080p, B 8, late passes,
    against the oracle's own mesh DFS on a row subset."""
    sc = big_mesh4
    W, H, first, S, B = 1920, 1080, 6_145, 2, 8
    renderer.set_traversal(traversal)
    try:
        img = render(mcpt_mod, renderer, sc, W, H, first, S, B)
    finally:
        renderer.set_traversal(0)
    rows = np.arange(13, H, 151)
    prims, nodes, leaves = sc.buffers()
    ipv, iv = oracle_mod.camera(W, H)
    mv = oracle_mod.MeshView(sc.mesh_buffers())
    for y in rows:
        ref, _ = oracle_mod.render(prims, nodes, leaves, sc.depth(), ipv, iv, W, H, first, S, 0.0, B, 1.0, 0,
                                   row_step=H, row_offset=int(y), meshes=mv)
        assert np.array_equal(bits(img[y]), bits(ref[int(y)])), f"four-mesh scene row {y}"
    assert np.isfinite(img).all() and img.mean() > 0


def test_mesh_big_split_items_same_bits(mcpt_mod, renderer, big_mesh4, monkeypatch):
    """Work-item order + split items on the four-mesh workload: three 64-pass calls equal the same
    passes in launch order without splits, bit for bit."""
    W, H, B = 1920, 1080, 8
    renderer.set_traversal(1)
    try:
        monkeypatch.setenv("MCPT_ITEM_ORDER", "1")
        a = render(mcpt_mod, renderer, big_mesh4, W, H, 1, 192, B, split=[64, 64, 64])
        n_split = int(renderer.debug_counters()[63])
        monkeypatch.setenv("MCPT_ITEM_ORDER", "0")
        b = render(mcpt_mod, renderer, big_mesh4, W, H, 1, 192, B, split=[64, 64, 64])
    finally:
        renderer.set_traversal(0)
    assert n_split > 0
    assert np.array_equal(bits(a), bits(b))
