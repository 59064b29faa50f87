"""Fuzz: the product's host scene producer (libmcpt, mcpt_scene.cpp) vs the oracle's
independent restatement on random scenes — record layout, emissive-first order, BVH nodes
and leaves bit for bit (the 8 reference scenes are covered by test_host_producer.py)."""
import numpy as np
import pytest

from fuzz_scenes import build_product, random_ops


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("seed", range(64))
def test_random_scene_buffers(mcpt_mod, oracle_mod, seed):
    ops = random_ops(mcpt_mod, seed)
    s = build_product(mcpt_mod, ops)
    prims, nodes, leaves = s.buffers()
    oprims, onodes, oleaves, odepth, oemi = oracle_mod.custom_scene(ops)
    assert s.depth() == odepth and s.nb_emissives() == oemi and s.nb_prim() == len(ops)
    assert np.array_equal(leaves.reshape(-1), oleaves)
    assert np.array_equal(bits(nodes).reshape(-1), bits(onodes).reshape(-1))
    # the inverse (texels 4-7) is Eigen's float inverse in the reference; both sides use
    # their own restatement of it, which agree on these well-conditioned transforms
    assert np.array_equal(bits(prims).reshape(-1), bits(oprims).reshape(-1))
