"""HIP kernel (through the C ABI) vs the CPU oracle, same inputs, same seeds.

Bar: bit-exact accumulators.  The kernel and the oracle implement the same binary32
arithmetic contract, so every pixel of every pass must agree to the bit;
the north-star tolerance (per-pixel RGB within 1e-3 of the reference integrator at equal
spp) is asserted as well, as a floor, with the mismatch statistics in the message.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-3   # north_star: per-pixel RGB within 1e-3 at equal spp


@pytest.fixture(scope="module")
def renderer(mcpt_mod):
    r = mcpt_mod.Renderer(0)
    yield r
    r.close()


def _gpu(mcpt_mod, r, scene_id, W, H, first, S, B, ior=1.0, variant=0, li=1.2, band_rows=8, world=1, rank=0,
         scene=None, split=None, traversal=0):
    sc = scene if scene is not None else mcpt_mod.Scene.reference(scene_id, li)
    r.set_traversal(traversal)
    r.upload_scene(sc)
    r.set_target(W, H, band_rows, world, rank)
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    chunks = split or [S]
    p = first
    for n in chunks:
        r.render(ipv, iv, p, n, 0.0, B, ior, variant)
        p += n
    acc, npass = r.read_accum()
    assert npass == S
    return acc


def _oracle(orc, scene_id, W, H, first, S, B, ior=1.0, variant=0, li=1.2, bufs=None, row_step=1, row_offset=0):
    prims, nodes, leaves, d, _ = bufs if bufs is not None else orc.scene(scene_id, li)
    ipv, iv = orc.camera(W, H)
    acc, ev = orc.render(prims, nodes, leaves, d, ipv, iv, W, H, first, S, 0.0, B, ior, variant,
                         row_step=row_step, row_offset=row_offset)
    return acc, ev


def _compare(gpu, ref, what):
    assert gpu.shape == ref.shape, what
    same = gpu.view(np.uint32) == ref.view(np.uint32)
    n_bad = int((~same).sum())
    diff = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
    assert np.isfinite(gpu).all(), f"{what}: non-finite output"
    assert n_bad == 0, (f"{what}: {n_bad}/{same.size} channels differ; max |diff| {diff.max():.3g} "
                        f"at {np.unravel_index(diff.argmax(), diff.shape)}")
    assert diff.max() <= TOL


TRAVERSALS = [1, 2, 3]   # MCPT_TRAVERSAL_LANE, _WAVE, _STREAM: same bits required from all


@pytest.mark.parametrize("traversal", TRAVERSALS)
@pytest.mark.parametrize("scene_id,B", [(1, 3), (2, 8), (3, 8), (4, 8), (5, 8), (6, 8), (7, 8), (8, 12)])
def test_scene_parity(mcpt_mod, oracle_mod, renderer, scene_id, B, traversal):
    W, H, S = 64, 48, 3
    gpu = _gpu(mcpt_mod, renderer, scene_id, W, H, 1, S, B, traversal=traversal)
    ref, _ = _oracle(oracle_mod, scene_id, W, H, 1, S, B)
    _compare(gpu, ref, f"scene {scene_id} traversal {traversal}")


@pytest.mark.parametrize("traversal", TRAVERSALS)
@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("scene_id", [1, 6, 8])
def test_variant_parity(mcpt_mod, oracle_mod, renderer, scene_id, variant, traversal):
    W, H, S = 48, 40, 2
    gpu = _gpu(mcpt_mod, renderer, scene_id, W, H, 1, S, 3, variant=variant, traversal=traversal)
    ref, _ = _oracle(oracle_mod, scene_id, W, H, 1, S, 3, variant=variant)
    _compare(gpu, ref, f"scene {scene_id} variant {variant} traversal {traversal}")


def test_auto_traversal_resolution(mcpt_mod, renderer):
    """AUTO resolves per scene depth (kWaveMaxDepth) and can be overridden."""
    renderer.set_traversal(0)
    for sid in (6, 8):
        renderer.upload_scene(mcpt_mod.Scene.reference(sid))
        assert renderer.traversal() in (1, 2)
    renderer.set_traversal(1)
    assert renderer.traversal() == 1
    renderer.set_traversal(0)


@pytest.mark.parametrize("traversal", TRAVERSALS)
def test_ior_and_light(mcpt_mod, oracle_mod, renderer, traversal):
    gpu = _gpu(mcpt_mod, renderer, 6, 64, 36, 5, 3, 8, ior=1.5, li=0.443, traversal=traversal)
    ref, _ = _oracle(oracle_mod, 6, 64, 36, 5, 3, 8, ior=1.5, li=0.443)
    _compare(gpu, ref, "scene 6 ior 1.5 light 0.443")


@pytest.mark.parametrize("rough", [0.0, 0.5, 0.9, 0.99, 1.0])
def test_roughness_sweep(mcpt_mod, oracle_mod, renderer, rough):
    """C3: override mat.g of the ground and the 4 spheres (emissive light unchanged)."""
    sc = mcpt_mod.Scene.reference(6)
    prims, nodes, leaves = sc.buffers()
    for i in range(sc.nb_prim()):
        rec = prims[i]
        if rec[58] > 0:
            continue
        m = np.concatenate([rec[52:56], [rec[56], rough, rec[58]]]).astype(np.float32)
        sc.set_material(i, m)
    prims2, _, _ = sc.buffers()
    gpu = _gpu(mcpt_mod, renderer, 6, 48, 32, 1, 3, 8, ior=1.5, scene=sc)
    ref, _ = _oracle(oracle_mod, 6, 48, 32, 1, 3, 8, ior=1.5, bufs=(prims2, nodes, leaves, sc.depth(), 1))
    _compare(gpu, ref, f"roughness {rough}")


def test_zero_bounces_is_black(mcpt_mod, renderer):
    gpu = _gpu(mcpt_mod, renderer, 6, 32, 16, 1, 2, 0)
    assert (gpu == 0).all()


def test_multi_launch_equals_single(mcpt_mod, renderer):
    """Calls split at multiples of the 32-pass accumulation chunk give identical sums."""
    one = _gpu(mcpt_mod, renderer, 2, 24, 16, 1, 70, 4)
    split = _gpu(mcpt_mod, renderer, 2, 24, 16, 1, 70, 4, split=[32, 32, 6])
    assert np.array_equal(one.view(np.uint32), split.view(np.uint32))


@pytest.mark.parametrize("budget_segments", [1, 2, 3])
@pytest.mark.parametrize("first,S", [(1, 200), (20, 150), (7, 33)])
def test_partial_budget_split_bit_equal(mcpt_mod, oracle_mod, renderer, budget_segments, first, S):
    """A call spanning more chunks than the segment-sum budget holds runs as several launches
    cut at chunk boundaries: same bits as one launch and as the oracle, same event counts."""
    W, H, B = 24, 16, 4
    ref, ev_ref = _oracle(oracle_mod, 6, W, H, first, S, B)
    one = _gpu(mcpt_mod, renderer, 6, W, H, first, S, B)
    assert renderer.last_launch_count() == 1
    renderer.set_partial_budget(budget_segments * W * H * 12)
    try:
        split = _gpu(mcpt_mod, renderer, 6, W, H, first, S, B)
        chunks = (first + S - 2) // 32 - (first - 1) // 32 + 1
        assert renderer.last_launch_count() == -(-chunks // budget_segments)
        tr, cb = renderer.last_kernel_ms()
        assert tr > 0.0 and cb >= 0.0
        ipv, iv = mcpt_mod.camera_canonical(W, H)
        ev = renderer.render_counted(ipv, iv, first, S, 0.0, B, 1.0, 0)
    finally:
        renderer.set_partial_budget(1 << 30)
    assert np.array_equal(one.view(np.uint32), split.view(np.uint32))
    _compare(split, ref, f"split passes {first}..{first + S - 1}")
    assert np.array_equal(ev, ev_ref), (ev, ev_ref)


@pytest.mark.parametrize("traversal", [1, 2])
@pytest.mark.parametrize("scene_id,B", [(1, 3), (6, 8), (8, 12)])
@pytest.mark.parametrize("first,S", [(1, 4), (30, 5), (1, 40), (7, 100), (33, 2)])
def test_pass_split_bit_equal(mcpt_mod, oracle_mod, renderer, monkeypatch, traversal, scene_id, B, first, S):
    """Pass split (one segment per pass, the split combine summing each chunk's passes in order)
    against the unsplit launch and the oracle, with pass ranges that start inside a chunk and
    straddle chunk boundaries."""
    W, H = 40, 24
    monkeypatch.setenv("MCPT_PASS_SPLIT", "0")
    whole = _gpu(mcpt_mod, renderer, scene_id, W, H, first, S, B, traversal=traversal)
    assert not renderer.last_pass_split()
    monkeypatch.setenv("MCPT_PASS_SPLIT", "1")
    split = _gpu(mcpt_mod, renderer, scene_id, W, H, first, S, B, traversal=traversal)
    assert renderer.last_pass_split()
    assert renderer.last_launch_count() == 1
    assert np.array_equal(whole.view(np.uint32), split.view(np.uint32))
    ref, _ = _oracle(oracle_mod, scene_id, W, H, first, S, B)
    _compare(split, ref, f"pass split scene {scene_id} passes {first}..{first + S - 1}")


def test_pass_split_default_small_launch(mcpt_mod, renderer, monkeypatch):
    """Without the override, a launch with few work items per CU splits, a large one does not."""
    monkeypatch.delenv("MCPT_PASS_SPLIT", raising=False)
    _gpu(mcpt_mod, renderer, 1, 256, 256, 1, 4, 3, traversal=1)   # C1's shape: 256 tiles
    assert renderer.last_pass_split()
    _gpu(mcpt_mod, renderer, 6, 1920, 1080, 1, 2, 8, traversal=1)  # 8,160 tiles
    assert not renderer.last_pass_split()
    _gpu(mcpt_mod, renderer, 1, 256, 256, 1, 1, 3, traversal=1)   # one pass: nothing to split
    assert not renderer.last_pass_split()


@pytest.mark.parametrize("first,S", [(20, 50), (1, 64), (33, 1), (7, 100)])
def test_pass_segments_vs_oracle(mcpt_mod, oracle_mod, renderer, first, S):
    """Launches spanning several accumulation chunks (segment sums + combine kernel)."""
    gpu = _gpu(mcpt_mod, renderer, 6, 16, 12, first, S, 4)
    ref, _ = _oracle(oracle_mod, 6, 16, 12, first, S, 4)
    _compare(gpu, ref, f"passes {first}..{first + S - 1}")


@pytest.mark.parametrize("world,band_rows", [(2, 8), (3, 4), (8, 8)])
def test_row_band_shards_bit_equal(mcpt_mod, renderer, world, band_rows):
    W, H = 40, 53
    full = _gpu(mcpt_mod, renderer, 6, W, H, 1, 2, 8, band_rows=band_rows)
    for rank in range(world):
        part = _gpu(mcpt_mod, renderer, 6, W, H, 1, 2, 8, band_rows=band_rows, world=world, rank=rank)
        rows = renderer.local_row_ids()
        assert part.shape[0] == len(rows)
        assert np.array_equal(part.view(np.uint32), full[rows].view(np.uint32))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_balanced_shards_bit_equal(mcpt_mod, renderer, world):
    """mcpt_set_target_rows with the balanced partition (and a reversed row list): each
    local row equals the full-frame render's row, bit for bit."""
    from mcpt.dist import local_rows
    W, H = 40, 53
    full = _gpu(mcpt_mod, renderer, 6, W, H, 1, 2, 8)
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    for rank in range(world):
        for rows in (local_rows(H, 8, world, rank, "balanced"), local_rows(H, 8, world, rank, "balanced")[::-1]):
            renderer.set_target_rows(W, H, rows)
            assert np.array_equal(renderer.local_row_ids(), rows)
            renderer.render(ipv, iv, 1, 2, 0.0, 8, 1.0, 0)
            part, n = renderer.read_accum()
            assert n == 2 and part.shape[0] == len(rows)
            assert np.array_equal(part.view(np.uint32), full[rows].view(np.uint32))


@pytest.mark.parametrize("traversal", TRAVERSALS)
@pytest.mark.parametrize("scene_id,B", [(6, 8), (8, 12), (7, 8), (1, 3)])
def test_event_counters_match_oracle(mcpt_mod, oracle_mod, renderer, scene_id, B, traversal):
    W, H, S = 40, 30, 2
    sc = mcpt_mod.Scene.reference(scene_id)
    renderer.set_traversal(traversal)
    renderer.upload_scene(sc)
    renderer.set_target(W, H, 8, 1, 0)
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    ev = renderer.render_counted(ipv, iv, 1, S, 0.0, B, 1.0, 0)
    _, ref_ev = _oracle(oracle_mod, scene_id, W, H, 1, S, B)
    renderer.set_traversal(0)
    assert np.array_equal(ev, ref_ev), (ev, ref_ev)


@pytest.mark.parametrize("traversal", TRAVERSALS)
def test_full_hd_rows_subset(mcpt_mod, oracle_mod, renderer, traversal):
    """C2 geometry at full size: 1920x1080, B=8; oracle checks every 45th row."""
    W, H, S, B = 1920, 1080, 2, 8
    gpu = _gpu(mcpt_mod, renderer, 6, W, H, 1, S, B, traversal=traversal)
    assert np.isfinite(gpu).all() and (gpu >= 0).all()
    ref, _ = _oracle(oracle_mod, 6, W, H, 1, S, B, row_step=45, row_offset=7)
    rows = np.arange(7, H, 45)
    _compare(gpu[rows], ref[rows], "1080p scene 6 row subset")


def test_golden_fixtures(mcpt_mod, renderer):
    """Kernel vs the committed oracle images (tests/golden/img_*.npy), bit-exact."""
    import os
    import sys
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, gold)
    import gen_golden as g
    for c in g.IMAGES:
        s, v, W, H, p, n, B, ior, li = c
        gpu = _gpu(mcpt_mod, renderer, s, W, H, p, n, B, ior=ior, variant=v, li=li)
        _compare(gpu, np.load(os.path.join(gold, g.image_name(c))), g.image_name(c))


def test_sharded_renderer_single_rank(mcpt_mod):
    """mcpt.dist.ShardedRenderer at world 1: torch-stream launch + D2D copy path."""
    import torch
    from mcpt.dist import ShardedRenderer
    W, H = 48, 32
    sr = ShardedRenderer(W, H, 8, 1, 0, 0)
    sr.upload_scene(mcpt_mod.Scene.reference(6))
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    sr.render(ipv, iv, 1, 3, 0.0, 8, 1.0, 0)
    frame = sr.gather()
    torch.cuda.synchronize()
    acc, _ = sr.r.read_accum()
    sr.close()
    assert np.array_equal(frame.cpu().numpy().view(np.uint32), acc.view(np.uint32))


@pytest.mark.parametrize("walk_exit", [0, 8, 40])
@pytest.mark.parametrize("scene_id,B,variant,ior", [(6, 8, 0, 1.5), (3, 8, 0, 1.0), (2, 5, 0, 1.3), (6, 4, 2, 1.0)])
def test_walk_exit_parity(mcpt_mod, oracle_mod, renderer, walk_exit, scene_id, B, variant, ior):
    """Suspended per-lane walks (mcpt_set_walk_exit) change only the interleaving: bit-exact."""
    W, H, S = 48, 40, 5
    renderer.set_walk_exit(walk_exit)
    try:
        gpu = _gpu(mcpt_mod, renderer, scene_id, W, H, 3, S, B, ior=ior, variant=variant, traversal=1)
        assert renderer.walk_exit() == walk_exit
    finally:
        renderer.set_walk_exit(-1)
    ref, _ = _oracle(oracle_mod, scene_id, W, H, 3, S, B, ior=ior, variant=variant)
    _compare(gpu, ref, f"scene {scene_id} walk_exit {walk_exit}")


@pytest.mark.parametrize("walk_exit,leaf_batch", [(0, 8), (16, 1), (16, 64), (24, 8), (0, 0)])
@pytest.mark.parametrize("scene_id,B,ior", [(3, 8, 1.0), (8, 6, 1.5), (6, 8, 1.5)])
def test_leaf_batch_parity(mcpt_mod, oracle_mod, renderer, walk_exit, leaf_batch, scene_id, B, ior):
    """Batched leaf visits (mcpt_set_leaf_batch) with and without suspension: bit-exact."""
    W, H, S = 40, 32, 3
    renderer.set_walk_exit(walk_exit)
    renderer.set_leaf_batch(leaf_batch)
    try:
        gpu = _gpu(mcpt_mod, renderer, scene_id, W, H, 7, S, B, ior=ior, traversal=1)
        assert renderer.leaf_batch() == leaf_batch
    finally:
        renderer.set_walk_exit(-1)
        renderer.set_leaf_batch(-1)
    ref, _ = _oracle(oracle_mod, scene_id, W, H, 7, S, B, ior=ior)
    _compare(gpu, ref, f"scene {scene_id} walk_exit {walk_exit} leaf_batch {leaf_batch}")


def test_auto_traversal_tuning(mcpt_mod, renderer):
    """AUTO times LANE then WAVE on the first two sizeable launches (then both again, in reverse)
    and keeps the faster one; the image is bit-identical to a fixed strategy with the same launch
    split."""
    W, H = 1920, 1080
    ipv, iv = mcpt_mod.camera_canonical(W, H)

    def run(mode):
        renderer.set_traversal(mode)          # also restarts the AUTO measurement
        renderer.upload_scene(mcpt_mod.Scene.reference(6))
        renderer.set_target(W, H)
        seen = []
        for k in range(3):                    # 1080p x 16 passes = 33 M samples >= 2^24
            seen.append(renderer.traversal())
            renderer.render(ipv, iv, 1 + 16 * k, 16, 0.0, 4, 1.0, 0)
        seen.append(renderer.traversal())
        acc, n = renderer.read_accum()
        return acc, n, seen

    auto, n_a, seen = run(0)
    lane, n_l, _ = run(1)
    renderer.set_traversal(0)
    # (the candidate the NEXT launch runs: LANE, WAVE, then round 2 in reverse order, WAVE, LANE)
    assert seen[:3] == [1, 2, 2] and seen[3] in (1, 2)
    assert n_a == n_l == 48
    assert np.array_equal(auto.view(np.uint32), lane.view(np.uint32))



@pytest.mark.parametrize("k", [2, 3, 5])
@pytest.mark.parametrize("first,S", [(1, 160), (17, 100)])
def test_segments_per_item_bit_equal(mcpt_mod, oracle_mod, renderer, monkeypatch, k, first, S):
    """Work items of k consecutive pass segments (MCPT_SEG_PER_ITEM; AUTO's candidate 3 runs
    k = 2): each segment's sum is written when its chunk ends — bits equal to one segment per
    item and to the oracle."""
    ref, _ = _oracle(oracle_mod, 6, 24, 16, first, S, 8)
    monkeypatch.setenv("MCPT_SEG_PER_ITEM", "1")
    one = _gpu(mcpt_mod, renderer, 6, 24, 16, first, S, 8, traversal=1)
    monkeypatch.setenv("MCPT_SEG_PER_ITEM", str(k))
    for trav in TRAVERSALS:
        gpu = _gpu(mcpt_mod, renderer, 6, 24, 16, first, S, 8, traversal=trav)
        assert np.array_equal(gpu.view(np.uint32), one.view(np.uint32)), (k, trav)
    _compare(one, ref, f"passes {first}..{first + S - 1}, {k} segments per item")


def test_auto_schedule_three_candidates(mcpt_mod, renderer):
    """On a launch of 8 pass segments (1080p x 256 passes) AUTO times four candidates
    (per-lane, wave-coherent, per-lane with two and with four segments per work item) before
    it settles; the image equals a fixed per-lane render."""
    W, H, S = 1920, 1080, 256
    ipv, iv = mcpt_mod.camera_canonical(W, H)

    def run(mode):
        renderer.set_traversal(mode)
        renderer.upload_scene(mcpt_mod.Scene.reference(6))
        renderer.set_target(W, H)
        seen = []
        for k in range(4):
            seen.append(renderer.traversal())
            renderer.render(ipv, iv, 1 + S * k, S, 0.0, 3, 1.0, 0)
        seen.append(renderer.traversal())
        acc, n = renderer.read_accum()
        return acc, n, seen

    auto, n_a, seen = run(0)
    lane, n_l, _ = run(1)
    renderer.set_traversal(0)
    # (the traversal of the NEXT launch: trials LANE, WAVE, then the two- and four-segment per-lane
    # candidates; then round 2 in reverse order)
    assert seen[:4] == [1, 2, 1, 1] and seen[4] in (1, 2), seen
    assert n_a == n_l == 4 * S
    assert np.array_equal(auto.view(np.uint32), lane.view(np.uint32))


def test_set_target_rows_rejects_bad_rows(mcpt_mod, renderer):
    """mcpt_set_target_rows: rows must be distinct and inside [0, H)."""
    for rows in ([0, 1, 1], [0, 5], [-1, 2]):
        with pytest.raises(mcpt_mod.MCPTError):
            renderer.set_target_rows(8, 5, rows)
    renderer.set_target_rows(8, 5, [4, 0])
    assert renderer.local_row_ids().tolist() == [4, 0]
    # a shard of 2^31 pixels or more is refused before any allocation (the kernels index a
    # shard's pixels with 32-bit ints); the context keeps its target
    with pytest.raises(mcpt_mod.MCPTError):
        renderer.set_target(1 << 16, 1 << 15)
    assert renderer.local_row_ids().tolist() == [4, 0]


def test_empty_and_tiny_shards(mcpt_mod, renderer):
    """More ranks than rows (H = 5, world = 8): the balanced partition leaves some ranks with no
    rows; those render nothing and read back an empty accumulator, the others match the frame."""
    from mcpt.dist import local_rows
    W, H = 40, 5
    full = _gpu(mcpt_mod, renderer, 6, W, H, 1, 2, 8)
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    for rank in range(8):
        rows = local_rows(H, 8, 8, rank, "balanced")
        renderer.set_target_rows(W, H, rows)
        renderer.render(ipv, iv, 1, 2, 0.0, 8, 1.0, 0)
        part, n = renderer.read_accum()
        assert n == 2 and part.shape == (len(rows), W, 3)
        assert np.array_equal(part.view(np.uint32), full[rows].view(np.uint32))


@pytest.mark.parametrize("world", [1, 3, 8])
def test_gather_rows_assembles_frame(mcpt_mod, world):
    """mcpt_gather_rows: shard contexts (balanced partition; one with its row list reversed)
    copied into a full-frame context equal the one-context render bit for bit; the frame's
    pass count is the shards'; bad arguments fail with a status, not silently."""
    W, H, S, B = 37, 45, 3, 8
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    sc = mcpt_mod.Scene.reference(6)
    full = mcpt_mod.Renderer(0)
    full.upload_scene(sc)
    full.set_target(W, H)
    full.render(ipv, iv, 1, S, 0.0, B, 1.0, 0)
    ref, n_ref = full.read_accum()
    shards = []
    for rank in range(world):
        r = mcpt_mod.Renderer(0)
        r.upload_scene(sc)
        from mcpt import dist
        rows = [int(y) for y in np.nonzero(dist.balanced_owner(H, 8, world) == rank)[0]]
        if rank == world - 1:
            rows = rows[::-1]
        r.set_target_rows(W, H, rows)
        r.render(ipv, iv, 1, S, 0.0, B, 1.0, 0)
        shards.append(r)
    frame = mcpt_mod.Renderer(0)
    frame.set_target(W, H)
    frame.gather_rows(shards)
    got, n = frame.read_accum()
    assert n == n_ref == S
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    if world > 1:
        with pytest.raises(mcpt_mod.MCPTError):
            shards[0].gather_rows(shards[1:])   # a shard is not a full-frame target
    other = mcpt_mod.Renderer(0)
    other.set_target(W + 1, H)
    with pytest.raises(mcpt_mod.MCPTError):
        other.gather_rows(shards)               # frame size differs from the shards'
    for r in shards + [frame, full, other]:
        r.close()


@pytest.mark.gpu
def test_gather_rows_then_render_again(mcpt_mod):
    """A progressive caller: render, gather_rows, render again at once, then read the frame.
    The shards' next renders add into their accumulators in place; they must wait for the peer
    copies of the gather (mcpt_gather_rows orders each shard's stream after them), so the frame
    holds exactly the first pass range (= a one-context render of it) and its pass count."""
    W, H, S1, S2, B = 640, 360, 32, 1024, 8
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    sc = mcpt_mod.Scene.reference(6)
    full = mcpt_mod.Renderer(0)
    full.upload_scene(sc)
    full.set_target(W, H)
    full.set_traversal(mcpt_mod.TRAVERSAL_LANE)
    full.render(ipv, iv, 1, S1, 0.0, B, 1.0, 0)
    ref, n_ref = full.read_accum()
    from mcpt import dist
    shards = []
    for rank in range(2):
        r = mcpt_mod.Renderer(0)
        r.upload_scene(sc)
        r.set_traversal(mcpt_mod.TRAVERSAL_LANE)
        r.set_target_rows(W, H, [int(y) for y in np.nonzero(dist.balanced_owner(H, 8, 2) == rank)[0]])
        shards.append(r)
    frame = mcpt_mod.Renderer(0)
    frame.set_target(W, H)
    for r in shards:
        r.render(ipv, iv, 1, S1, 0.0, B, 1.0, 0)
    frame.gather_rows(shards)
    for r in shards:   # queued right after the gather: must not reach the rows being copied
        r.render(ipv, iv, S1 + 1, S2, 0.0, B, 1.0, 0)
    got, n = frame.read_accum()
    assert n == n_ref == S1
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    for r in shards:
        _, ns = r.read_accum()
        assert ns == S1 + S2
    for r in shards + [frame, full]:
        r.close()


@pytest.mark.parametrize("scene_id,n_cand", [(6, 4), (8, 5)])
def test_auto_two_round_trials_settle(mcpt_mod, renderer, scene_id, n_cand):
    """AUTO times each applicable candidate twice (candidate order, then reverse) on launches of
    one shape and then settles (mcpt_get_schedule reports it); mcpt.AUTO_TRIALS launches are
    enough; the image equals a fixed per-lane render of the same launches.  Candidates: per-lane,
    wave-coherent (BVH depth < 8 only), per-lane with 2 and 4 segments per item, and (BVH depth
    >= 8: scene 8) the deep-knob walks at 4 and 8 segments per item.  The stream schedule is never
    timed by AUTO, nor is the wave-coherent walk on a deep BVH (its trial cost 8.4 s on C4)."""
    W, H, S = 1920, 1080, 256   # 8 pass segments: the segment-group candidates apply
    ipv, iv = mcpt_mod.camera_canonical(W, H)

    def run(mode, n):
        renderer.set_traversal(mode)
        renderer.upload_scene(mcpt_mod.Scene.reference(scene_id))
        renderer.set_target(W, H)
        sched = []
        for k in range(n):
            renderer.render(ipv, iv, 1 + S * k, S, 0.0, 3, 1.0, 0)
            sched.append(renderer.schedule())
        acc, cnt = renderer.read_accum()
        return acc, cnt, sched

    assert mcpt_mod.AUTO_TRIALS >= 2 * n_cand + 2
    auto, n_a, sched = run(0, mcpt_mod.AUTO_TRIALS + 1)
    # a trial's time is collected when the call after the next one starts (round 6: consecutive
    # trials overlap on the render lanes): settled after 2 * n_cand + 2 calls
    assert not any(s["settled"] for s in sched[:2 * n_cand + 1]), sched
    assert all(s["settled"] for s in sched[2 * n_cand + 1:]), sched
    assert sched[-1]["seg_per_item"] in (1, 2, 4, 8), sched
    tried = {s["traversal"] for s in sched[:2 * n_cand]}
    assert "stream" not in tried, sched
    assert ("wave" in tried) == (scene_id != 8), sched
    assert sched[-1]["traversal"] in (("lane",) if scene_id == 8 else ("lane", "wave"))
    lane, n_l, fixed = run(1, mcpt_mod.AUTO_TRIALS + 1)
    renderer.set_traversal(0)
    assert all(s["settled"] and s["traversal"] == "lane" for s in fixed)
    assert n_a == n_l
    assert np.array_equal(auto.view(np.uint32), lane.view(np.uint32))


def test_kernel_ms_back_ring(mcpt_mod, renderer):
    """mcpt_kernel_ms_back: the events of the last TIMING_RING calls are kept; a call further
    back (or before any call) is an error."""
    W, H = 64, 40
    renderer.set_traversal(1)
    renderer.upload_scene(mcpt_mod.Scene.reference(6))
    renderer.set_target(W, H)
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    for k in range(3):
        renderer.render(ipv, iv, 1 + 8 * k, 8 * (k + 1), 0.0, 8, 1.0, 0)   # 8, 16, 24 passes
    t = [renderer.kernel_ms_back(b)[0] for b in (2, 1, 0)]
    assert all(x > 0.0 for x in t)
    assert renderer.kernel_ms_back(0) == renderer.last_kernel_ms()
    with pytest.raises(RuntimeError):
        renderer.kernel_ms_back(mcpt_mod.Renderer.TIMING_RING)
    r2 = mcpt_mod.Renderer(0)
    try:
        with pytest.raises(RuntimeError):
            r2.kernel_ms_back(0)
    finally:
        r2.close()


@pytest.mark.gpu
@pytest.mark.parametrize("scene_id,traversal", [(6, 1), (8, 1), (3, 2)])
def test_item_order_same_bits(mcpt_mod, renderer, monkeypatch, scene_id, traversal):
    """The work-item order (mcpt_order.hip): launches of >= 4,096 items run their items
    costliest-first, sorted from the previous launch of the same shape.  Which workgroup runs an
    item never changes what it computes: three chunked calls (the first in launch order, the
    others in the measured order, one of them re-sorted) equal the same passes with the order
    off (MCPT_ITEM_ORDER=0), bit for bit (the unordered path is the one the oracle tests pin)."""
    W, H, B = 1920, 1080, 4
    chunks = [32, 32, 64]   # 8,100 tiles x 1-2 segments per launch
    monkeypatch.setenv("MCPT_ITEM_ORDER", "1")
    ordered = _gpu(mcpt_mod, renderer, scene_id, W, H, 1, 128, B, split=chunks, traversal=traversal)
    monkeypatch.setenv("MCPT_ITEM_ORDER", "0")
    plain = _gpu(mcpt_mod, renderer, scene_id, W, H, 1, 128, B, split=chunks, traversal=traversal)
    assert np.array_equal(ordered.view(np.uint32), plain.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("scene_id,traversal", [(6, 1), (8, 1)])
def test_tail_pieces_same_bits(mcpt_mod, renderer, monkeypatch, scene_id, traversal):
    """Items of several pass segments (MCPT_SEG_PER_ITEM=4): once ordered, the cheapest
    generation of items at the end of the order runs one segment per workgroup (tail pieces).
    Each segment still sums its passes from 0 into its own slot, so three 128-pass calls equal
    the same calls with the order off, bit for bit."""
    W, H, B = 1920, 1080, 4
    monkeypatch.setenv("MCPT_SEG_PER_ITEM", "4")
    monkeypatch.setenv("MCPT_ITEM_ORDER", "1")
    ordered = _gpu(mcpt_mod, renderer, scene_id, W, H, 1, 384, B, split=[128, 128, 128], traversal=traversal)
    monkeypatch.setenv("MCPT_ITEM_ORDER", "0")
    plain = _gpu(mcpt_mod, renderer, scene_id, W, H, 1, 384, B, split=[128, 128, 128], traversal=traversal)
    assert np.array_equal(ordered.view(np.uint32), plain.view(np.uint32))


@pytest.mark.parametrize("scene_id,B,traversal", [(6, 8, 1), (8, 12, 1), (3, 8, 2), (0, 8, 1)])
def test_render_lanes_same_bits(mcpt_mod, monkeypatch, scene_id, B, traversal):
    """Render lanes (round 6): once the schedule is settled, consecutive launches alternate between
    two lanes (streams, segment-sum buffers, work-item order state), each render starting while
    the previous one's last workgroups run; the combines stay in call order.  Four 96-pass calls,
    then one 384-pass call cut into four sub-launches by a small segment-sum budget (lanes
    alternate inside a call), equal the same calls with the lanes off (MCPT_OVERLAP=0, every launch
    in order on one stream), bit for bit.  Scene 0: the mesh workload (split items per lane)."""
    W, H = (960, 540) if scene_id else (1920, 1080)
    if scene_id == 0:
        from mcpt import meshes
        sc = meshes.big_mesh_scene(1_000_000)[0]
    else:
        sc = mcpt_mod.Scene.reference(scene_id)
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    out = {}
    for ov in ("1", "0"):
        monkeypatch.setenv("MCPT_OVERLAP", ov)
        r = mcpt_mod.Renderer(0)
        try:
            r.set_traversal(traversal)
            r.upload_scene(sc)
            r.set_target(W, H)
            p = 1
            for _ in range(4):
                r.render(ipv, iv, p, 96, 0.0, B, 1.0, 0)
                p += 96
            a, n = r.read_accum()
            r.clear_accum()
            r.set_partial_budget(W * H * 12 * 3)   # three segments per sub-launch
            r.render(ipv, iv, 1, 384, 0.0, B, 1.0, 0)
            launches = r.last_launch_count()
            b, n2 = r.read_accum()
        finally:
            r.close()
        assert n == 384 and n2 == 384 and launches == 4
        out[ov] = (a, b)
    for k in range(2):
        assert np.array_equal(out["1"][k].view(np.uint32), out["0"][k].view(np.uint32)), (scene_id, k)
