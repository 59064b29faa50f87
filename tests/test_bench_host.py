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


def test_pmc_record_by_schedule(tmp_path, monkeypatch):
    """Records of one workload under two schedules sit side by side; the run's own schedule picks
    its record, and a schedule with no record gets one whose schedule roofline() then rejects."""
    s2 = {"traversal": "lane", "seg_per_item": 2}
    s4 = {"traversal": "lane", "seg_per_item": 4}
    recs = {"records": [
        {"workload": "scene6_1920x1080_256spp_B8", "lib_sha256": "aa", "schedule": s4, "counters_per_launch": {"SQ_INSTS_VALU": 4}},
        {"workload": "scene6_1920x1080_256spp_B8", "lib_sha256": "aa", "schedule": s2, "counters_per_launch": {"SQ_INSTS_VALU": 2}},
    ]}
    f = tmp_path / "pmc_records.json"
    f.write_text(json.dumps(recs))
    monkeypatch.setattr(bench, "PMC_RECORDS", str(f))
    w = "scene6_1920x1080_256spp_B8"
    assert bench.pmc_record(w, "aa", dict(s2, settled=True))["counters_per_launch"]["SQ_INSTS_VALU"] == 2
    assert bench.pmc_record(w, "aa", s4)["counters_per_launch"]["SQ_INSTS_VALU"] == 4
    roof = bench.roofline(w, "aa", 10.0, 1e9, 100.0, 1, sched={"traversal": "wave", "seg_per_item": 2})
    assert roof["pmc"]["matched"] is False and roof["frac"] is None
    roof = bench.roofline(w, "aa", 10.0, 1e9, 100.0, 1, sched=dict(s2, settled=True))
    assert roof["pmc"]["matched"] is True and roof["valu_instructions_per_launch"] == 2


def test_pmc_summary_keeps_other_schedules():
    """tools/pmc_summary.py's merge: a new record replaces its own (workload, schedule) slot only;
    a mixed-schedule record (None) takes the whole workload; other builds' records are dropped."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import importlib
    merge = importlib.import_module("pmc_summary").merge_record
    s2, s4 = {"traversal": "lane", "seg_per_item": 2}, {"traversal": "lane", "seg_per_item": 4}
    w, v = "scene6_1920x1080_256spp_B8", "scene8_1920x1080_512spp_B12"
    def r(wl, sc, sha="aa", tag=0):
        return {"workload": wl, "lib_sha256": sha, "schedule": sc, "tag": tag}
    recs = merge([r(w, s4, tag=1), r(v, s4), r(w, s4, sha="old")], r(w, s2, tag=2))
    assert sorted((x["workload"], x["schedule"]["seg_per_item"], x["tag"]) for x in recs) == \
        [(w, 2, 2), (w, 4, 1), (v, 4, 0)]
    recs = merge(recs, r(w, s4, tag=3))                 # same slot: replaced
    assert sorted(x["tag"] for x in recs if x["workload"] == w) == [2, 3]
    recs = merge(recs, r(w, None, tag=4))               # mixed schedules: the workload's only record
    assert [x["tag"] for x in recs if x["workload"] == w] == [4]
    recs = merge(recs, r(w, s2, tag=5))                 # and a settled one replaces it
    assert [x["tag"] for x in recs if x["workload"] == w] == [5]


def test_mesh_roofline_fabric_request_ceiling(tmp_path, monkeypatch):
    """The mesh workloads' `limiter` prices the PMC fabric requests per second against the measured
    ceiling of their access pattern (tools/microbench/gather_ceiling.hip), keyed by the workload."""
    rec = {"workload": "mesh4x1000k_1920x1080_64spp_B8", "lib_sha256": "aa", "launches_summed": 1,
           "counters_per_launch": {"SQ_INSTS_VALU": 1e9}, "hbm_bytes_per_launch": 4e11,
           "valu_lane_utilisation": 0.25, "memory": {"fabric_reads": 3.0e9}}
    f = tmp_path / "pmc_records.json"
    f.write_text(json.dumps({"records": [rec]}))
    monkeypatch.setattr(bench, "PMC_RECORDS", str(f))
    roof = bench.roofline("mesh4x1000k_1920x1080_64spp_B8", "aa", 100.0, 4e11, 3000.0, 1, bound="hbm")
    c = roof["limiter"]["fabric_request_ceiling"]
    assert c["walk_requests_per_s"] == 30.0                      # 3 G requests in 100 ms
    assert c["frac"] == round(30e9 / bench.GATHER_CEILING_REQ_S["mesh4x1000k"], 4)
    # a workload without a measured ceiling (or a record without memory counters) carries none
    rec["workload"] = "mesh999k_1920x1080_64spp_B8"
    f.write_text(json.dumps({"records": [rec]}))
    roof = bench.roofline("mesh999k_1920x1080_64spp_B8", "aa", 100.0, 4e11, 3000.0, 1, bound="hbm")
    assert "fabric_request_ceiling" not in roof["limiter"]


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


def test_cpu_baseline_reports_the_faster_run(monkeypatch):
    """The CPU baseline runs one worker per CPU of the affinity mask and, when the cgroup quota
    grants fewer CPUs' time, one per granted CPU; `value` is the faster run, `cores` its thread
    count, the other run beside it (verdict r04 #4, advisor r04).  A bounded C1 sample keeps this
    a quick CPU test."""
    args = bench.parse(["--config", "c1"])
    cb = bench.cpu_baseline(args, 0.2)
    avail = len(os.sched_getaffinity(0))
    assert cb["cores_available"] == avail and cb["cgroup_cpu_quota"] == bench.cpu_quota()
    assert cb["threads_used"] == cb["cores"] and cb["value"] > 0 and cb["kind"] == "port"
    assert "primary hit" in cb["algorithm_note"]
    # a quota below the mask: two runs, the faster one is the value
    fake = {2: 5.0, 1: 7.0}
    monkeypatch.setattr(bench, "cpus_available", lambda: 2)
    monkeypatch.setattr(bench, "cpu_quota", lambda: 1.0)
    monkeypatch.setattr(bench, "cpu_baseline_run",
                        lambda a, s, rough=None, threads=None, scene=None:
                        {"value": fake[threads], "threads": threads, "sample": f"t{threads}", "nproc": 2, "model": "x"})
    cb = bench.cpu_baseline(args, 1.0)
    assert cb["value"] == 7.0 and cb["cores"] == 1 and cb["threads_used"] == 1
    assert cb["other_runs"] == [{"threads": 2, "value": 5.0, "sample": "t2"}]
    fake[2] = 9.0
    cb = bench.cpu_baseline(args, 1.0)
    assert cb["value"] == 9.0 and cb["cores"] == 2 and cb["other_runs"][0]["threads"] == 1


def test_stall_report_names_least_advanced_rank():
    import time
    now = time.time()
    last = {0: ("stats", now), 1: ("timed", now - 5), 2: ("stats", now)}
    rep = bench.stall_report(last, {1, 2}, 3)
    assert "Stalled: rank(s) 1 in phase timed (next: stats)" in rep
    assert "rank 0 exited, last phase stats" in rep and "rank 1 running" in rep
    rep = bench.stall_report({0: ("auto", now)}, {0, 1}, 2)      # rank 1 never stamped
    assert "Stalled: rank(s) 1 in phase (no stamp yet)" in rep
    assert bench.parse_stamp("bench-phase rank=3 phase=gather t=1.5") == (3, "gather")
    assert bench.parse_stamp("other line") is None


def _drill_env():
    env = dict(os.environ, MCPT_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    return env


def test_drill_stalled_rank_is_named_within_the_deadline():
    """Verdict r04 #2: `bench.py --gpus 2` with one rank stalling before a phase exits non-zero
    inside its deadline and names that rank and phase (gloo, CPU only: --drill-stall walks the
    phases with collectives and no GPU work)."""
    import subprocess
    import time
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--deadline", "15",
                        "--drill-stall", "1:stats"], env=_drill_env(), capture_output=True, text=True, timeout=120)
    dt = time.time() - t0
    assert p.returncode != 0 and "{" not in p.stdout         # no result line
    assert dt < 15 + 15 + 20, dt
    assert "Stalled: rank(s) 1 in phase timed (next: stats)" in p.stderr, p.stderr[-2000:]
    assert "bench-phase rank=0 phase=stats" in p.stderr


def test_drill_success_relays_the_line():
    import subprocess
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--deadline", "60",
                        "--drill-stall", "1:cpu_baseline:0.2"], env=_drill_env(), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["drill"] is True and d["n_gpus"] == 2
    assert p.stderr.count("phase=done") == 2


def test_default_multi_gpu_run_is_strong_scaling():
    """`bench.py --gpus N` (the driver's N-GPU command) renders ONE fixed C2 frame split N ways
    (verdict r05 #4); weak scaling is the opt-in.  The gloo rehearsal of the default 2-rank run
    reports it in its line."""
    import subprocess
    for argv, want in ((["--gpus", "2"], "strong"), (["--gpus", "8", "--config", "c3"], "strong"),
                       (["--gpus", "2", "--scaling", "weak"], "weak"), (["--config", "c4"], "strong")):
        assert bench.parse(argv).scaling == want, argv
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--deadline", "60",
                        "--drill-stall", "1:done:0"], env=_drill_env(), capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 2 and d["config"] == "c2" and d["scaling"] == "strong"


def test_deadline_default_and_off():
    a = bench.parse([])
    assert a.deadline == 600.0 + 30.0 * (a.steps + a.warmup)
    assert bench.parse(["--config", "c3", "--steps", "2", "--warmup", "1"]).deadline == 600.0 + 30.0 * 3 * 5
    assert bench.parse(["--deadline", "0"]).deadline is None
    assert bench.parse(["--deadline", "42"]).deadline == 42.0


def test_drill_rank_deadline_under_torchrun():
    """Launched by torch.distributed.run (the driver's N-GPU command), a rank past --deadline
    names its phase and exits 124 by itself."""
    import subprocess
    import time
    t0 = time.time()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(bench.free_port()),
                        os.path.join(REPO, "bench.py"), "--gpus", "2", "--deadline", "10", "--drill-stall",
                        "0:count"], env=_drill_env(), capture_output=True, text=True, timeout=150)
    assert p.returncode != 0
    assert time.time() - t0 < 90
    # whichever rank's watchdog fires first names its phase: rank 0 sleeps before `count` (its
    # phase: stats), rank 1 waits for it in the `count` barrier
    import re
    assert re.search(r"bench rank (0: deadline 10 s reached in phase stats|1: deadline 10 s reached in phase count)",
                     p.stderr), p.stderr[-2000:]


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
