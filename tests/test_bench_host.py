"""Host-side logic of bench.py (CPU): the self-check row choice covers every rank's shard, and
PMC records are only used for the exact library build they were measured on."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

import bench  # noqa: E402
from mcpt.dist import balanced_owner  # noqa: E402


def test_check_rows_cover_every_rank():
    for world in (1, 2, 3, 8):
        rows = bench.check_rows(1080, 8, world)
        owners = set(balanced_owner(1080, 8, world)[rows].tolist())
        assert owners == set(range(world)), (world, owners)
        assert rows == sorted(set(rows)) and rows[-1] == 1079


def test_pmc_record_keyed_by_library_hash(tmp_path, monkeypatch):
    recs = {"records": [
        {"workload": "scene6_1920x1080_256spp_B8", "lib_sha256": "aa", "counters_per_launch": {"SQ_INSTS_VALU": 1}},
        {"workload": "scene8_1920x1080_512spp_B12", "lib_sha256": "aa", "counters_per_launch": {"SQ_INSTS_VALU": 2}},
    ]}
    f = tmp_path / "pmc_records.json"
    f.write_text(json.dumps(recs))
    monkeypatch.setattr(bench, "PMC_RECORDS", str(f))
    assert bench.pmc_record("scene6_1920x1080_256spp_B8", "aa")["counters_per_launch"]["SQ_INSTS_VALU"] == 1
    assert bench.pmc_record("scene8_1920x1080_512spp_B12", "aa")["counters_per_launch"]["SQ_INSTS_VALU"] == 2
    assert bench.pmc_record("scene6_1920x1080_256spp_B8", "bb") is None      # other build: never used
    assert bench.pmc_record("scene6_1920x1080_512spp_B8", "aa") is None      # other workload
    monkeypatch.setattr(bench, "PMC_RECORDS", str(tmp_path / "missing.json"))
    assert bench.pmc_record("scene6_1920x1080_256spp_B8", "aa") is None


def test_workload_keys():
    class A:
        scene, width, height, bounces = 6, 1920, 1080, 8
    assert bench.workload_key(A, 256) == "scene6_1920x1080_256spp_B8"
    for name, c in bench.CONFIGS.items():
        assert c["scaling"] in ("weak", "strong")
    assert bench.CONFIGS["c2"]["scene"] == 6 and bench.CONFIGS["c4"]["scene"] == 8
    assert np.isclose(bench.VALU_PEAK_T, 256 * 4 * 32 * 2.4e9 / 1e12, rtol=1e-3)
