"""Random scenes for the fuzz tests: primitives of every analytic type under random affine
transforms (translations, rotations about x/y/z, non-uniform scales) with random materials
(opaque / translucent, shininess, roughness, some emissive), built identically through the
product's scene producer (mcpt.Scene) and the oracle's (oracle.custom_scene)."""
import numpy as np

ADD = {1: "add_sphere", 2: "add_cube", 3: "add_cylinder", 4: "add_cone", 5: "add_oriented_quad"}


def random_ops(mcpt_mod, seed, n_min=1, n_max=40):
    rng = np.random.default_rng(seed)
    T = mcpt_mod.Transfo
    n = int(rng.integers(n_min, n_max + 1))
    ops = []
    for k in range(n):
        t = int(rng.integers(1, 6))
        trf = T.mul(T.translate(*rng.uniform(-120, 120, 3).round(2)),
                    T.rotateZ(float(rng.uniform(0, 360))), T.rotateX(float(rng.uniform(0, 360))),
                    T.rotateY(float(rng.uniform(0, 360))),
                    T.scale(*rng.uniform(2, 45, 3).round(2)))
        col = [*rng.uniform(0, 1, 3).round(3), 1.0 if rng.random() < 0.5 else float(rng.uniform(0.02, 0.98))]
        shin = 0.0 if rng.random() < 0.3 else float(rng.uniform(0.05, 1.0))
        rough = float(rng.uniform(0, 1))
        emi = float(rng.uniform(1, 30)) if (k == 0 or rng.random() < 0.1) else 0.0
        ops.append((t, trf, np.array(col + [shin, rough, emi], np.float32)))
    if rng.random() < 0.7:   # a ground slab under most scenes
        ops.append((2, T.mul(T.translate(0, 0, -140), T.scale(400, 400, 2)),
                    np.array([0.8, 0.8, 0.8, 1.0, 0.2, 0.9, 0.0], np.float32)))
    return ops


def build_product(mcpt_mod, ops):
    s = mcpt_mod.Scene()
    for t, trf, mat in ops:
        getattr(s, ADD[t])(trf, mat)
    s.finalize()
    return s
