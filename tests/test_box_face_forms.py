"""The kernel's rewritten box-test / primitive-test conditions equal the reference's forms.

`box_face` (csrc/mcpt_device.h) tests a face's two in-face bounds as one compare of their
NaN-propagating maximum (v_maximum3_f32), where intersect_bv (raytracer_func.frag:314-352)
writes `abs(p) <= 1 && abs(q) <= 1`; the inside test the same way with `< 1`.  numpy's
`np.maximum` propagates NaN like `llvm.maximum`, so the identities are checked here over the
float32 values that matter (signed zeros, denormals, the bounds and their neighbours,
infinities, NaN) and a random sample; the GPU parity suites check the kernels themselves.
"""
import numpy as np

F32 = np.float32


def _specials():
    one = F32(1.0)
    v = [0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1e-10, 3.402823e38,
         np.nextafter(one, F32(2)), np.nextafter(one, F32(0)),
         -np.nextafter(one, F32(2)), -np.nextafter(one, F32(0)), 0.5, -0.5, 2.0, -2.0]
    return np.array(v, dtype=F32)


def _pairs():
    s = _specials()
    p, q = np.meshgrid(s, s)
    rng = np.random.default_rng(4)
    r = (rng.standard_normal((2, 200000)) * 1.2).astype(F32)
    return np.concatenate([p.ravel(), r[0]]), np.concatenate([q.ravel(), r[1]])


def test_maximum_le_equals_both_le():
    p, q = _pairs()
    with np.errstate(invalid="ignore"):
        ref = (np.abs(p) <= 1) & (np.abs(q) <= 1)
        got = np.maximum(np.abs(p), np.abs(q)) <= 1
    assert np.array_equal(ref, got)


def test_maximum_lt_equals_all_lt():
    p, q = _pairs()
    r = np.roll(p, 7)
    with np.errstate(invalid="ignore"):
        ref = (np.abs(p) < 1) & (np.abs(q) < 1) & (np.abs(r) < 1)
        got = np.maximum(np.maximum(np.abs(p), np.abs(q)), np.abs(r)) < 1
    assert np.array_equal(ref, got)


def test_maxnum_is_wrong_for_nan():
    """Why the NaN-propagating maximum: fmax (maxNum) drops a NaN and accepts the face."""
    with np.errstate(invalid="ignore"):
        assert not (np.abs(F32(np.nan)) <= 1)
        assert np.fmax(np.abs(F32(np.nan)), F32(0.5)) <= 1
        assert not (np.maximum(np.abs(F32(np.nan)), F32(0.5)) <= 1)


def _faces_min(cands, valid, first_plain):
    """intersect_bv's `if (a < al) al = a` from FLT_MAX (reference) or the kernel's min chain."""
    kmax = F32(3.402823e38)
    al = kmax
    for i, (a, ok) in enumerate(zip(cands, valid)):
        if first_plain and i == 0:
            al = a if ok else kmax
        else:
            al = min(al, a if ok else kmax)
    return al


def test_first_face_without_min_keeps_the_result():
    """MCPT_FACE_FIRST: the first candidate taken as is changes al only above kFLTMAX."""
    kmax = F32(3.402823e38)
    vals = [F32(0.5), F32(2.0), kmax, F32(np.inf), np.nextafter(kmax, F32(np.inf)), F32(1e-9)]
    rng = np.random.default_rng(1)
    for _ in range(3000):
        cands = [vals[i] for i in rng.integers(0, len(vals), 6)]
        valid = rng.integers(0, 2, 6).astype(bool)
        ref = _faces_min(cands, valid, False)
        got = _faces_min(cands, valid, True)
        assert (ref < kmax) == (got < kmax)
        if ref < kmax:
            assert ref == got
