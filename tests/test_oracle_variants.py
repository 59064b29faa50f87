"""What "per-pixel RGB within 1e-3 of the GLSL reference at equal spp" means while parity with
the executed reference stays unpinned (the reference needs a GL 4.3 context,
Eigen, GLFW and assimp, none of which exist here).

The shipped arithmetic contract fixes every piece the reference leaves implementation-defined.
Each deviation below swaps in ONE such piece as a real GL driver or Eigen build might have it
(oracle.cpp DEV_*), and measures how far the averaged image moves against the shipped oracle
(= the HIP kernel, bit for bit):

* DEV_TC_UP / DEV_TC_DOWN — the interpolated ``screen_tc`` whose float bits seed the RNG
  (raytracer_func.frag:105-110) one ulp up / down: a different rasterizer interpolation;
* DEV_LIBM — libm ``sinf/cosf/logf/powf`` instead of the contract polynomials (driver
  transcendental precision, tp/montecarlo.frag:61-67, 134);
* DEV_DIV — true divisions in ``intersect_bv`` (raytracer_func.frag:322-335) instead of the
  reciprocal multiplications a GLSL compiler emits;
* DEV_INV_F32 — a binary32 Gauss-Jordan 4x4 inverse instead of the double adjugate for the
  primitive inverses (scene.cpp:48, Eigen's float ``inverse()``) and the camera
  (montecarlo.cpp:439-440).

Crops: C2 (scene 6, 1080p frame, 256 spp, B 8, IOR 1.0) and C3 (scene 6, 1024 spp, B 8,
IOR 1.5, roughness 0.5 on every non-emissive primitive), 64×48 pixels each, rendered by the
CPU oracle.  Figures go to profiles/r03_parity_variants.json (deterministic: no timings).
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as orc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "profiles", "r03_parity_variants.json")
W, H = 1920, 1080
CROP = (928, 520, 64, 48)   # x0, y0 (row 0 = bottom), w, h: spheres, ground and sky edges
BAR = 1e-3                  # the north star's per-pixel RGB tolerance

CASES = {
    "C2": dict(spp=256, bounces=8, ior=1.0, rough=None),
    "C3": dict(spp=1024, bounces=8, ior=1.5, rough=0.5),
}
DEVIATIONS = {
    "screen_tc_plus_1ulp": orc.DEV_TC_UP,
    "screen_tc_minus_1ulp": orc.DEV_TC_DOWN,
    "libm_sin_cos_log_pow": orc.DEV_LIBM,
    "true_division_intersect_bv": orc.DEV_DIV,
    "float_gauss_jordan_inverse": orc.DEV_INV_F32,
}


def crop_xy():
    x0, y0, w, h = CROP
    xs, ys = np.meshgrid(np.arange(x0, x0 + w), np.arange(y0, y0 + h))
    return np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)


def render_avg(case, flags):
    c = CASES[case]
    with orc.deviation(flags):
        prims, nodes, leaves, depth, _ = orc.scene(6)
        ipv, iv = orc.camera(W, H)
        if c["rough"] is not None:
            prims = prims.copy()
            prims[~(prims[:, 58] > 0), 57] = c["rough"]
        acc = orc.render_pixels(prims, nodes, leaves, depth, ipv, iv, W, H, crop_xy(), 1, c["spp"], 0.0,
                                c["bounces"], c["ior"], 0)
    return acc / np.float32(c["spp"])


@pytest.fixture(scope="module")
def baselines():
    return {case: render_avg(case, 0) for case in CASES}


def stats(a, b):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64)).max(axis=1)   # per pixel, max over RGB
    return {"max_abs": float(d.max()), "mean_abs": float(d.mean()), "p99_abs": float(np.quantile(d, 0.99)),
            "frac_pixels_over_1e-3": float((d > BAR).mean()), "pixels_identical": int((d == 0).sum())}


def test_deviation_zero_is_the_contract(baselines):
    for case in CASES:
        again = render_avg(case, 0)
        assert np.array_equal(again.view(np.uint32), baselines[case].view(np.uint32))


def test_parity_variants_figures(baselines):
    out = {"what": "per-pixel |delta| (max over RGB) of the averaged image against the shipped oracle "
                   "(= the HIP kernel bit for bit), one implementation-defined piece swapped at a time",
           "crop": {"x0": CROP[0], "y0_from_bottom": CROP[1], "w": CROP[2], "h": CROP[3], "frame": [W, H]},
           "bar": BAR, "cases": {}}
    res = {}
    for case, c in CASES.items():
        base = baselines[case]
        entry = {"config": c, "mean_pixel_value": float(base.mean()), "max_pixel_value": float(base.max()),
                 "deviations": {}}
        for name, flags in DEVIATIONS.items():
            st = stats(render_avg(case, flags), base)
            entry["deviations"][name] = st
            res[(case, name)] = st
        # Monte Carlo noise at this spp for scale: the same pixels with the next spp passes
        with orc.deviation(0):
            prims, nodes, leaves, depth, _ = orc.scene(6)
            ipv, iv = orc.camera(W, H)
            if c["rough"] is not None:
                prims = prims.copy()
                prims[~(prims[:, 58] > 0), 57] = c["rough"]
            other = orc.render_pixels(prims, nodes, leaves, depth, ipv, iv, W, H, crop_xy(), c["spp"] + 1, c["spp"],
                                      0.0, c["bounces"], c["ior"], 0) / np.float32(c["spp"])
        entry["mc_noise_other_passes"] = stats(other, base)
        out["cases"][case] = entry
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    for case in CASES:
        # the driver's transcendental precision and the compiler's division form stay inside
        # the 1e-3 bar everywhere on the crops (true division changed no box decision here)
        assert 0 < res[(case, "libm_sin_cos_log_pow")]["max_abs"] < BAR, case
        assert res[(case, "true_division_intersect_bv")]["max_abs"] < BAR, case
        # a different float inverse moves hit points by ulps: tiny on average, but a path whose
        # branch flips can move a pixel by ~1e-3 (C2: one pixel just above the bar)
        inv = res[(case, "float_gauss_jordan_inverse")]
        assert inv["max_abs"] > 0 and inv["mean_abs"] < 1e-4 and inv["frac_pixels_over_1e-3"] < 0.01, case
        # a seed that differs in one bit is a different Monte Carlo sample: the difference is
        # the estimator's noise, far above the 1e-3 bar at 256 / 1024 spp
        noise = out["cases"][case]["mc_noise_other_passes"]["mean_abs"]
        for name in ("screen_tc_plus_1ulp", "screen_tc_minus_1ulp"):
            assert res[(case, name)]["max_abs"] > BAR and res[(case, name)]["frac_pixels_over_1e-3"] > 0.5
            assert 0.5 * noise < res[(case, name)]["mean_abs"] < 2 * noise
