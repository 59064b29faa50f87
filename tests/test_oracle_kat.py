"""Pin the CPU oracle against the golden known-answer vectors (tests/golden/kat.npz).

The vectors come from an independent numpy float32 restatement of the GLSL pieces
(tests/golden/gen_golden.py), so a coding slip in oracle.cpp shows up here as a bit
mismatch.  Bar: bit-exact (integer hashes, binary32 values).
"""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def kat():
    return dict(np.load(os.path.join(GOLD, "kat.npz")))


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def test_xxhash32(oracle_mod, kat):
    out = np.array([oracle_mod.xxhash32(*map(int, x)) for x in kat["xx_in"]], np.uint32)
    assert np.array_equal(out, kat["xx_out"])


def test_srand_and_random_float(oracle_mod, kat):
    for i, (tc, p, d) in enumerate(zip(kat["srand_in"], kat["srand_pass"], kat["srand_date"])):
        seed = oracle_mod.srand(float(tc[0]), float(tc[1]), int(p), float(d))
        assert np.array_equal(seed, kat["srand_seed"][i]), i
        seq = oracle_mod.random_floats(seed, 16)
        assert np.array_equal(bits(seq), bits(kat["rf_seq"][i])), i
        assert ((seq >= 0) & (seq < 1)).all()


def test_sincos(oracle_mod, kat):
    out = np.array([oracle_mod.sincos(float(x)) for x in kat["sc_in"]], np.float32)
    assert np.array_equal(bits(out), bits(kat["sc_out"]))
    ref = np.stack([np.sin(kat["sc_in"].astype(np.float64)), np.cos(kat["sc_in"].astype(np.float64))], 1)
    assert np.abs(out - ref).max() < 4e-7     # contract accuracy: a few ulp on [0, 2pi)


def test_log_exp2_pow(oracle_mod, kat):
    L = oracle_mod.lib()
    lo = np.array([L.orc_log(float(x)) for x in kat["log_in"]], np.float32)
    assert np.array_equal(bits(lo), bits(kat["log_out"]))
    ex = np.array([L.orc_exp2(float(x)) for x in kat["exp2_in"]], np.float32)
    assert np.array_equal(bits(ex), bits(kat["exp2_out"]))
    pw = np.array([L.orc_pow(float(a), float(b)) for a, b in kat["pow_in"]], np.float32)
    assert np.array_equal(bits(pw), bits(kat["pow_out"]))
    x = kat["log_in"][np.isfinite(kat["log_in"]) & (kat["log_in"] > 1e-37)].astype(np.float64)
    rel = np.abs(np.array([L.orc_log(float(v)) for v in x]) - np.log(x)) / np.maximum(np.abs(np.log(x)), 1e-6)
    assert rel.max() < 1e-6


def test_random_ray_sampler(oracle_mod, kat):
    for d, s, r, want in zip(kat["rr_dir"], kat["rr_seed"], kat["rr_rough"], kat["rr_out"]):
        out, _ = oracle_mod.random_ray(s, d, float(r))
        assert np.array_equal(bits(out), bits(want)), (d, s, r)
        assert abs(np.linalg.norm(out.astype(np.float64)) - 1) < 1e-6
        if r == 0:
            assert np.allclose(out, d, atol=1e-6)    # roughness 0: the lobe collapses to D


def test_intersect_prim(oracle_mod, kat):
    n = len(kat["ip_rec"])
    hits = 0
    for i in range(n):
        shape, dist, dr, pl, pg = oracle_mod.intersect_prim(kat["ip_rec"][i], kat["ip_O"][i], kat["ip_D"][i])
        assert shape == kat["ip_shape"][i], i
        assert bits(dist) == bits(kat["ip_dist"][i]), i
        if shape >= 0:
            hits += 1
            assert dr == kat["ip_dir"][i], i
            assert np.array_equal(bits(pl), bits(kat["ip_pl"][i])), i
            assert np.array_equal(bits(pg), bits(kat["ip_pg"][i])), i
    assert hits > n // 4   # the generator aims rays at the primitives


def test_golden_images(oracle_mod):
    import sys
    sys.path.insert(0, GOLD)
    import gen_golden as g
    for c in g.IMAGES:
        s, v, W, H, p, n, B, ior, li = c
        pr, nodes, leaves, d, _ = oracle_mod.scene(s, li)
        ipv, iv = oracle_mod.camera(W, H)
        acc, _ = oracle_mod.render(pr, nodes, leaves, d, ipv, iv, W, H, p, n, 0.0, B, ior, v)
        want = np.load(os.path.join(GOLD, g.image_name(c)))
        assert np.array_equal(bits(acc), bits(want)), c


def test_cone_intersect(oracle_mod, kat):
    """Cone_intersect (raytracer_func.frag:579-640) vs the numpy restatement; cones accept
    backward roots (no a > EPSILON check on the lateral surface), kept."""
    n = len(kat["cone_rec"])
    hits = 0
    for i in range(n):
        shape, dist, dr, pl, pg = oracle_mod.intersect_prim(kat["cone_rec"][i], kat["cone_O"][i], kat["cone_D"][i])
        assert shape == kat["cone_shape"][i], i
        assert bits(dist) == bits(kat["cone_dist"][i]), i
        if shape >= 0:
            hits += 1
            assert dr == kat["cone_dir"][i], i
            assert np.array_equal(bits(pl), bits(kat["cone_pl"][i])), i
            assert np.array_equal(bits(pg), bits(kat["cone_pg"][i])), i
    assert hits > n // 4


def test_sampler_point_cloud(oracle_mod, kat):
    """DrawSampling seeding (tp/sampling_base.vert:23-26) + random_ray, bit-exact."""
    for nrm, fs, r, nb, want in zip(kat["smp_normal"], kat["smp_fseed"], kat["smp_rough"], kat["smp_nb"],
                                    kat["smp_out"]):
        got = oracle_mod.sample_hemisphere(nrm, fs, len(want), float(r), int(nb))
        assert np.array_equal(bits(got), bits(want))
        n = nrm / np.linalg.norm(nrm)
        if r > 0:
            assert (got @ n > 0).all()            # the lobe stays in the upper hemisphere


def test_any_hit_queries(oracle_mod):
    """just_hit_bvh finds a hit exactly when traverse_all_bvh does, never closer; one-prim
    queries agree with the closest hit on that primitive."""
    rng = np.random.default_rng(5)
    for sid in (1, 6, 8):
        prims, nodes, leaves, d, _ = oracle_mod.scene(sid)
        o = rng.uniform(-250, 250, (400, 3)).astype(np.float32)
        dd = rng.normal(size=(400, 3)).astype(np.float32)
        ci, cf = oracle_mod.trace(prims, nodes, leaves, d, o, dd)
        ai, af = oracle_mod.trace(prims, nodes, leaves, d, o, dd, any_hit=True)
        assert np.array_equal(ci[:, 0] >= 0, ai[:, 0] >= 0)
        hit = ci[:, 0] >= 0
        assert (af[hit, 0] >= cf[hit, 0]).all()
        assert hit.sum() > 20
        k = int(ci[hit][0, 1])
        pi, pf = oracle_mod.trace(prims, nodes, leaves, d, o, dd, prim=k)
        same = hit & (ci[:, 1] == k)
        assert np.array_equal(bits(pf[same]), bits(cf[same]))
