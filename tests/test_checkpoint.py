"""Checkpoint / resume of a progressive render (mcpt.h mcpt_checkpoint_write / _read,
mcpt_write_accum; mcpt_render --checkpoint / --resume).  The reference's pass loop
(MontecarloGPU/montecarlo.cpp:454-466) accumulates for as long as its window is open; a resumed
render here must give the bits of the uninterrupted one with the same render calls."""
import os
import subprocess

import numpy as np
import pytest

from test_cpp_host import read_pfm

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(REPO, "montecarlo-pathtracing_amd", "bin", "mcpt_render")


def test_checkpoint_file_roundtrip(mcpt_mod, tmp_path):
    rng = np.random.default_rng(5)
    acc = rng.standard_normal((7, 13, 3)).astype(np.float32)
    acc[0, 0] = [np.nan, np.inf, -0.0]
    p = str(tmp_path / "a.ckpt")
    mcpt_mod.checkpoint_write(p, acc, 96, 97, "scene=6 bounces=8")
    assert sorted(f.name for f in tmp_path.iterdir()) == ["a.ckpt"]   # no temporary file left
    back, n, nxt, tag = mcpt_mod.checkpoint_read(p)
    assert np.array_equal(back.view(np.uint32), acc.view(np.uint32))
    assert (n, nxt, tag) == (96, 97, "scene=6 bounces=8")
    # a later checkpoint replaces the file whole
    mcpt_mod.checkpoint_write(p, acc[:2], 128, 129)
    back, n, nxt, tag = mcpt_mod.checkpoint_read(p)
    assert back.shape == (2, 13, 3) and (n, nxt, tag) == (128, 129, "")


def test_checkpoint_rejects_bad_files(mcpt_mod, tmp_path):
    acc = np.ones((4, 5, 3), np.float32)
    p = str(tmp_path / "a.ckpt")
    mcpt_mod.checkpoint_write(p, acc, 1, 2, "t")
    data = open(p, "rb").read()
    cut = str(tmp_path / "cut.ckpt")
    open(cut, "wb").write(data[:-4])                     # truncated sums
    foreign = str(tmp_path / "foreign.ckpt")
    open(foreign, "wb").write(b"PF\n5 4\n-1.0\n" + data[12:])
    for bad in (cut, foreign, str(tmp_path / "missing.ckpt")):
        with pytest.raises(mcpt_mod.MCPTError):
            mcpt_mod.checkpoint_read(bad)
    # the reader never writes more than the caller's capacity (a file replaced between the
    # header read and the sums read)
    small = np.zeros(4 * 5 * 3 - 1, np.float32)
    assert mcpt_mod.lib().mcpt_checkpoint_read(p.encode(), mcpt_mod._fp(small), small.size,
                                               None, None, None, None, None) == -1
    assert mcpt_mod.lib().mcpt_checkpoint_read(p.encode(), mcpt_mod._fp(small), -1, None, None, None, None, None) == -1
    with pytest.raises(mcpt_mod.MCPTError):               # tag longer than the format allows
        mcpt_mod.checkpoint_write(p, acc, 1, 2, "x" * mcpt_mod.CHECKPOINT_TAG_MAX)
    with pytest.raises(mcpt_mod.MCPTError):
        mcpt_mod.checkpoint_write(str(tmp_path / "no_dir" / "a.ckpt"), acc, 1, 2)


def test_app_refuses_checkpoint_with_devices():
    if not os.path.exists(APP):
        pytest.skip("mcpt_render not built")
    r = subprocess.run([APP, "--devices", "0,0", "--checkpoint", "x.ckpt"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 2 and "--checkpoint" in r.stderr      # usage, before any GPU call


@pytest.mark.gpu
def test_resume_bit_equal_to_uninterrupted(mcpt_mod, tmp_path):
    """Passes 1..32 in one context, checkpoint, passes 33..64 in a fresh context after the
    load == passes 1..32 then 33..64 in one context, bit for bit; mismatched tag / shape raise."""
    W, H, B = 96, 64, 8
    sc = mcpt_mod.Scene.reference(6)
    ipv, iv = mcpt_mod.camera_canonical(W, H)

    def renderer():
        r = mcpt_mod.Renderer(0)
        r.upload_scene(sc)
        r.set_target(W, H)
        return r

    a = renderer()
    for first in (1, 33):
        a.render(ipv, iv, first, 32, 0.0, B, 1.0, mcpt_mod.MONTECARLO)
    want, n_want = a.read_accum()
    p = str(tmp_path / "s6.ckpt")
    b1 = renderer()
    b1.render(ipv, iv, 1, 32, 0.0, B, 1.0, mcpt_mod.MONTECARLO)
    b1.save_checkpoint(p, 33, "scene=6")
    b2 = renderer()
    nxt = b2.load_checkpoint(p, "scene=6")
    assert nxt == 33 and b2.read_accum()[1] == 32
    b2.render(ipv, iv, nxt, 32, 0.0, B, 1.0, mcpt_mod.MONTECARLO)
    got, n_got = b2.read_accum()
    assert n_got == n_want == 64
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    # call boundaries on the 32-pass accumulation chunks: also one call over passes 1..64
    c = renderer()
    c.render(ipv, iv, 1, 64, 0.0, B, 1.0, mcpt_mod.MONTECARLO)
    assert np.array_equal(c.read_accum()[0].view(np.uint32), want.view(np.uint32))
    with pytest.raises(mcpt_mod.MCPTError, match="tag"):
        renderer().load_checkpoint(p, "scene=7")
    small = mcpt_mod.Renderer(0)
    small.upload_scene(sc)
    small.set_target(W // 2, H)
    with pytest.raises(mcpt_mod.MCPTError):
        small.load_checkpoint(p)


@pytest.mark.gpu
def test_checkpoint_refuses_other_shard_or_frame(mcpt_mod, tmp_path):
    """A checkpoint carries its target's identity (H and the row ids): a shard's file does not
    load into another shard with the same row count, nor into a taller frame whose shard has the
    same local size, nor does a file written without identity (mcpt_checkpoint_write) load into a
    context (advisor r03)."""
    W, H = 64, 48
    sc = mcpt_mod.Scene.reference(6)
    ipv, iv = mcpt_mod.camera_canonical(W, H)

    def shard(h, rows):
        r = mcpt_mod.Renderer(0)
        r.upload_scene(sc)
        r.set_target_rows(W, h, rows)
        return r

    rows0, rows1 = list(range(0, H, 2)), list(range(1, H, 2))   # same local row count
    a = shard(H, rows0)
    a.render(ipv, iv, 1, 4, 0.0, 8, 1.0, mcpt_mod.MONTECARLO)
    p = str(tmp_path / "shard0.ckpt")
    a.save_checkpoint(p, 5, "s6")
    assert shard(H, rows0).load_checkpoint(p, "s6") == 5
    with pytest.raises(mcpt_mod.MCPTError, match="another target or shard"):
        shard(H, rows1).load_checkpoint(p, "s6")
    with pytest.raises(mcpt_mod.MCPTError, match="another target or shard"):
        shard(2 * H, rows0).load_checkpoint(p, "s6")
    raw = str(tmp_path / "raw.ckpt")
    acc, n = a.read_accum()
    mcpt_mod.checkpoint_write(raw, acc, n, 5, "s6")
    with pytest.raises(mcpt_mod.MCPTError, match="no target identity"):
        shard(H, rows0).load_checkpoint(raw, "s6")


@pytest.mark.gpu
def test_app_resume_matches_uninterrupted_and_oracle(oracle_mod, tmp_path):
    """mcpt_render --checkpoint after 4 of 6 passes, then --resume to 6 == one run of 6 passes
    with the same --chunk == the oracle's accumulation of the same launches."""
    W, H, B = 48, 40, 8
    base = [APP, "--scene", "6", "--width", str(W), "--height", str(H), "--chunk", "2", "--bounces", str(B)]
    one, res, ck = str(tmp_path / "one.pfm"), str(tmp_path / "res.pfm"), str(tmp_path / "s.ckpt")
    r = subprocess.run(base + ["--spp", "6", "--pfm", one], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    r = subprocess.run(base + ["--spp", "4", "--checkpoint", ck], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    r = subprocess.run(base + ["--spp", "6", "--resume", ck, "--pfm", res], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    a, b = read_pfm(one), read_pfm(res)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    prims, nodes, leaves, d, _ = oracle_mod.scene(6)
    ipv, iv = oracle_mod.camera(W, H)
    acc = np.zeros((H, W, 3), np.float32)
    for first in (1, 3, 5):
        oracle_mod.render(prims, nodes, leaves, d, ipv, iv, W, H, first, 2, 0.0, B, 1.0, 0, accum=acc)
    assert np.array_equal(b.view(np.uint32), (acc / np.float32(6)).view(np.uint32))
    # other render parameters: refused
    r = subprocess.run(base[:-2] + ["--bounces", "3", "--spp", "6", "--resume", ck], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 1 and "render parameters differ" in r.stderr
