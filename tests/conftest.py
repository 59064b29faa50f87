"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs on CPU (oracle vs golden vectors, host scene/BVH producer vs the
oracle's restatement, C-ABI symbol table, gloo multi-process sharding).  `-m gpu` runs
the HIP kernel through the C ABI against the oracle on a real MI355X.
"""
import os
import sys

import pytest
# torch first: its HIP runtime must be the process's one before libmcpt.so loads (as in
# bench.py), or torch.cuda finds no device in a session whose first HIP user was libmcpt
import torch  # noqa: F401,E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "montecarlo-pathtracing_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libmcpt.so")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as orc
    orc.lib()
    return orc


@pytest.fixture(scope="session")
def mcpt_mod():
    import mcpt
    mcpt.lib()
    return mcpt
