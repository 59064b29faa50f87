"""The oracle's integrator pinned to an independent restatement, sample by sample.

tests/golden/paths.npz holds 688 whole samples ((pixel, pass) at 1920×1080) of
tp/montecarlo.frag:100-179 computed by the numpy float32 restatement in
tests/golden/gen_golden.py (camera ray, intersect_bvh's literal stack DFS, intersect_bv,
the primitive tests, intersection_info, random_path with all four material branches, the
inner traversal and the exhausted-budget black), written from the GLSL text and the
arithmetic contract of DESIGN.md §3, not from oracle.cpp.  The cases cover all eight reference
scenes (6 and 5 also at IOR 1.5) and a scene with the pure-refraction branch no reference scene
reaches; 96 samples run the two other tp/ programs (montecarlo_mat.frag, montecarlo_mat_tr.frag:
one traversal, then abs(N)·random_vec3() or col.rgb·random_float()); each
case records the branch sequence its path took.  The oracle (and, in test_gpu_paths.py, the
HIP kernel) must reproduce every sample bit for bit.
"""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "paths.npz")


@pytest.fixture(scope="module")
def paths():
    return dict(np.load(GOLDEN, allow_pickle=False))


def scene_buffers(orc, kat, scene_id, light):
    if scene_id == 0:
        return kat["custom_prims"], kat["custom_nodes"], kat["custom_leaves"], int(kat["custom_depth"])
    prims, nodes, leaves, d, _ = orc.scene(int(scene_id), float(light))
    return prims, nodes, leaves, d


def test_branch_coverage(paths):
    codes = "".join(paths["path_trace"].tolist())
    # sky, emissive end, reflect, pure refraction, mixed reflect / refract, diffuse,
    # exhausted budget, inner traversal missing (N, P kept)
    for c in "SERTMmFXIV":
        assert codes.count(c) > 0, f"branch {c} not covered"
    assert set(paths["path_scene"].tolist()) == {0, 1, 2, 3, 4, 5, 6, 7, 8}
    assert set(paths["path_variant"].tolist()) == {0, 1, 2}   # montecarlo / _mat / _mat_tr
    assert len(paths["path_x"]) == 688


def test_oracle_matches_independent_paths(oracle_mod, paths):
    W, H = int(paths["path_W"]), int(paths["path_H"])
    ipv, iv = oracle_mod.camera(W, H)
    keys = sorted(set(zip(paths["path_scene"].tolist(), paths["path_light"].tolist(), paths["path_ior"].tolist(),
                          paths["path_bounces"].tolist(), paths["path_variant"].tolist())))
    n_checked = 0
    for scene_id, light, ior, B, variant in keys:
        sel = np.nonzero((paths["path_scene"] == scene_id) & (paths["path_light"] == np.float32(light)) &
                         (paths["path_ior"] == np.float32(ior)) & (paths["path_bounces"] == B) &
                         (paths["path_variant"] == variant))[0]
        prims, nodes, leaves, d = scene_buffers(oracle_mod, paths, scene_id, light)
        for i in sel:
            xy = np.array([[paths["path_x"][i], paths["path_y"][i]]], np.int32)
            got = oracle_mod.render_pixels(prims, nodes, leaves, d, ipv, iv, W, H, xy, int(paths["path_npass"][i]), 1,
                                           0.0, int(B), float(ior), int(variant), n_threads=1)[0]
            want = paths["path_rgb"][i]
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (
                f"scene {scene_id} variant {variant} ior {ior} B {B} pixel {tuple(xy[0])} pass {paths['path_npass'][i]} "
                f"branches {paths['path_trace'][i]}: oracle {got} vs restatement {want}")
            n_checked += 1
    assert n_checked == len(paths["path_x"])
