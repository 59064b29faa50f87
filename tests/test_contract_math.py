"""Identities the HIP kernel relies on to skip work while staying bit-exact (CPU check).

cull_bound_sq (mcpt_kernel.hip): for binary32 d2 >= 0 and c >= 0,
    RN32(sqrt(d2)) <= c   <=>   float64(d2) < m*m,   m = (c + nextafter(c, +inf)) / 2,
with m*m exact in binary64.  numpy's float32 sqrt is correctly rounded (IEEE), so this
checks the identity the box-test cull uses instead of the reference's sqrt
(raytracer_func.frag:351) on random and boundary cases.
"""
import numpy as np


def cull_bound_sq(c):
    c = np.asarray(c, np.float32)
    nx = (c.view(np.uint32) + np.uint32(1)).view(np.float32)
    m = (c.astype(np.float64) + nx.astype(np.float64)) * 0.5
    return m * m


def check(d2, c):
    d2 = np.asarray(d2, np.float32)
    c = np.asarray(c, np.float32)
    want = np.sqrt(d2) <= c
    got = d2.astype(np.float64) < cull_bound_sq(c)
    bad = want != got
    assert not bad.any(), (d2[bad][:5], c[bad][:5])


def test_random_magnitudes():
    rng = np.random.default_rng(1)
    e = rng.uniform(-30, 30, 2_000_000)
    d2 = (10.0 ** e).astype(np.float32)
    c = (np.sqrt(d2.astype(np.float64)) * rng.uniform(0.999, 1.001, d2.size)).astype(np.float32)
    check(d2, c)


def test_boundaries():
    rng = np.random.default_rng(2)
    c = (10.0 ** rng.uniform(-20, 20, 200_000)).astype(np.float32)
    # d2 values whose rounded sqrt lands exactly on c, or one float either side
    base = (c.astype(np.float64) ** 2).astype(np.float32)
    for k in range(-40, 41):
        d2 = (base.view(np.uint32).astype(np.int64) + k).clip(0, 0x7F7FFFFF).astype(np.uint32).view(np.float32)
        check(d2, c)


def test_specials():
    fmax = np.float32(3.402823e38)            # the kernel's initial cull distance
    check([0.0, 1e-45, 1.0, np.inf, np.nan, 3.4e38], [fmax] * 6)
    check([0.0, 1e-45, 0.0], [0.0, 0.0, 1e-45])
    check([np.inf, np.nan], [1.0, 1.0])
