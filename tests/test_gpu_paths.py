"""The HIP kernel against the independent integrator restatement (tests/golden/paths.npz, see
tests/test_oracle_paths.py): every one of the 688 (pixel, pass) samples (all three tp/ programs) at 1080p, rendered as a
one-pass launch of the sample's row through the C ABI, must equal the restatement bit for bit,
under every schedule (per-lane walk, wave-coherent walk, stream)."""
import numpy as np
import pytest

from test_oracle_paths import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("traversal", [1, 2, 3])   # MCPT_TRAVERSAL_LANE, _WAVE, _STREAM
def test_gpu_matches_independent_paths(mcpt_mod, traversal):
    kat = dict(np.load(GOLDEN, allow_pickle=False))
    W, H = int(kat["path_W"]), int(kat["path_H"])
    ipv, iv = mcpt_mod.camera_canonical(W, H)
    r = mcpt_mod.Renderer(0)
    bad = []
    try:
        r.set_traversal(traversal)
        current = None
        for i in range(len(kat["path_x"])):
            key = (int(kat["path_scene"][i]), float(kat["path_light"][i]))
            if key != current:
                if key[0] == 0:
                    prims = kat["custom_prims"]
                    r.upload_scene(prims=prims, nodes=kat["custom_nodes"], leaves=kat["custom_leaves"],
                                   depth=int(kat["custom_depth"]), nb_emissives=int((prims[:, 58] > 0).sum()))
                else:
                    r.upload_scene(mcpt_mod.Scene.reference(key[0], key[1]))
                current = key
            x, y = int(kat["path_x"][i]), int(kat["path_y"][i])
            r.set_target_rows(W, H, [y])
            r.render(ipv, iv, int(kat["path_npass"][i]), 1, 0.0, int(kat["path_bounces"][i]),
                     float(kat["path_ior"][i]), int(kat["path_variant"][i]))
            acc, n = r.read_accum()
            assert n == 1
            got, want = acc[0, x], kat["path_rgb"][i]
            if not np.array_equal(got.view(np.uint32), want.view(np.uint32)):
                bad.append((key, x, y, int(kat["path_npass"][i]), str(kat["path_trace"][i]), got.tolist(),
                            want.tolist()))
    finally:
        r.close()
    assert not bad, f"{len(bad)} samples differ, first: {bad[:3]}"
