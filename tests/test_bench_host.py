"""Host-side logic of bench.py (CPU): the self-check row choice covers every rank's shard, and
PMC records are only used for the exact library build they were measured on."""
import json
import os
import sys

import numpy as np
import pytest

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
    a = bench.parse(["--config", "c3", "--rough", "0.5"])
    assert bench.workload_key(a, 1024, 0.5) == "scene6_1920x1080_1024spp_B8_ior1.5_rough0.5"


def test_configs_match_baseline():
    """Every BASELINE.json config has a bench mode with its scene, size, spp and bounces."""
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))["configs"]
    want = {"c1": (1, 256, 256, 4, 3), "c2": (6, 1920, 1080, 256, 8), "c3": (6, 1920, 1080, 1024, 8),
            "c4": (8, 1920, 1080, 512, 12), "c5": (6, 3840, 2160, None, 8)}
    assert len(base) == len(want)
    for i, (k, (sc, w, h, spp, b)) in enumerate(sorted(want.items())):
        c = bench.CONFIGS[k]
        assert (c["scene"], c["width"], c["height"], c["bounces"]) == (sc, w, h, b), k
        assert f"{w}×{h}" in base[i] or f"{w}x{h}" in base[i] or (w == 256 and "256×256" in base[i])
        if spp is not None:
            assert c["spp"] == spp and f"{spp} spp" in base[i], k
    assert bench.CONFIGS["c3"]["ior"] == 1.5 and bench.CONFIGS["c3"]["rough_sweep"] == (0.0, 0.5, 0.9, 0.99, 1.0)
    assert bench.CONFIGS["c5"]["target_spp"] == 84000 and "84000 spp" in base[4]
    assert bench.parse(["--config", "c3"]).rough_points == (0.0, 0.5, 0.9, 0.99, 1.0)
    assert bench.parse(["--config", "c3", "--rough", "0.9"]).rough_points == (0.9,)
    assert bench.parse(["--config", "c2"]).rough_points == (None,)
    with pytest.raises(SystemExit):
        bench.parse(["--config", "c2", "--rough", "0.5"])


def test_check_world():
    assert bench.check_world(1, 1, "nccl", 1, 1) is None
    assert bench.check_world(8, 8, "nccl", 8, 8) is None
    assert "joined" in bench.check_world(8, 1, "nccl", 8, 1)      # plain run that did not spawn
    assert "joined" in bench.check_world(2, 4, "nccl", 8, 4)
    assert "visible" in bench.check_world(8, 8, "nccl", 1, 8)      # fewer GPUs than ranks (RCCL)
    assert bench.check_world(2, 2, "gloo", 1, 2) is None           # rehearsal: ranks share a GPU
    assert "no visible" in bench.check_world(1, 1, "gloo", 0, 1)


_CHILD = r"""
import json, os, sys, time
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
assert int(os.environ["MASTER_PORT"]) > 0
mode = sys.argv[1]
if mode == "fail" and r == w - 1:
    sys.exit(7)
if mode == "fail":
    time.sleep(60)      # would block in a collective: the launcher must stop it
if r == 0:
    print("noise")
    print(json.dumps({"n_gpus": w if mode != "short" else 1, "rank": r}))
"""


def test_spawn_ranks_env_and_rank0_line(tmp_path):
    child = tmp_path / "child.py"
    child.write_text(_CHILD)
    status, out = bench.spawn_ranks([sys.executable, str(child), "ok"], 3)
    assert status == 0
    line = bench.rank0_line(out, 3)
    assert line is not None and json.loads(line) == {"n_gpus": 3, "rank": 0}
    assert bench.rank0_line(out, 2) is None                 # a line for another world size: rejected
    status, out = bench.spawn_ranks([sys.executable, str(child), "short"], 2)
    assert status == 0 and bench.rank0_line(out, 2) is None


def test_spawn_ranks_failure_stops_the_others(tmp_path):
    import time
    child = tmp_path / "child.py"
    child.write_text(_CHILD)
    t0 = time.time()
    status, out = bench.spawn_ranks([sys.executable, str(child), "fail"], 3, grace_s=5.0)
    assert status == 7
    assert time.time() - t0 < 30                            # the sleeping ranks were stopped
    assert bench.rank0_line(out, 3) is None


def test_plain_gpus_n_launches_ranks_without_a_gpu_call(tmp_path, monkeypatch):
    """`bench.py --gpus N` with no WORLD_SIZE goes through launch(), whose children each get
    their rank; a child rejecting its world makes the launch fail with no line."""
    calls = []

    def fake_spawn(cmd, world, **kw):
        calls.append((cmd, world))
        return 3, ""
    monkeypatch.setattr(bench, "spawn_ranks", fake_spawn)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "1"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 3
    assert calls and calls[0][1] == 4 and calls[0][0][-4:] == ["--gpus", "4", "--steps", "1"]


def test_host_cpu_statement():
    n, model = bench.host_cpu()
    assert n == os.cpu_count()
    assert model is None or isinstance(model, str)
    assert bench.cpus_available() == len(os.sched_getaffinity(0))
    q = bench.cpu_quota()
    assert q is None or q > 0


def test_cpu_baseline_uses_available_cores():
    """The CPU baseline runs one worker per CPU of the process's affinity mask (verdict r03:
    not OMP_NUM_THREADS) and states it with the cgroup quota; a bounded C1 sample keeps this a
    quick CPU test."""
    args = bench.parse(["--config", "c1"])
    cb = bench.cpu_baseline(args, 0.2)
    avail = len(os.sched_getaffinity(0))
    assert cb["threads_used"] == cb["cores"] == cb["cores_available"] == avail
    assert cb["cgroup_cpu_quota"] == bench.cpu_quota()
    assert cb["value"] > 0 and cb["kind"] == "port"
    c1 = bench.cpu_baseline(args, 0.2, threads=1)
    assert c1["threads_used"] == 1


def test_cpu_threads_capped_by_quota(monkeypatch):
    monkeypatch.setattr(bench, "cpus_available", lambda: 256)
    monkeypatch.setattr(bench, "cpu_quota", lambda: 16.0)
    assert bench.cpu_threads() == 16
    monkeypatch.setattr(bench, "cpu_quota", lambda: 2.5)
    assert bench.cpu_threads() == 3
    monkeypatch.setattr(bench, "cpu_quota", lambda: None)
    assert bench.cpu_threads() == 256
    monkeypatch.setattr(bench, "cpus_available", lambda: 8)
    monkeypatch.setattr(bench, "cpu_quota", lambda: 64.0)
    assert bench.cpu_threads() == 8
