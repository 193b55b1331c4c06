"""Relation files (hj3d.relfile): reference-generator relations written once
and reloaded memory-mapped, bit-identical, with corruption and truncation detected."""
import os

import numpy as np
import pytest

import oracle as O
from hj3d import relfile


def exp1_rels(nR, nS):
    Rk, Sa, _ = O.gen_exp1(nR, nS, True, 0.8, 0)
    return O.tuples3(Rk, np.zeros_like(Rk)), O.tuples3(np.arange(nS, dtype=np.uint32), Sa)


def test_roundtrip_bit_exact(tmp_path, monkeypatch):
    monkeypatch.setattr(relfile, "CHUNK", 1000)  # several chunks
    R, S = exp1_rels(4096, 20000)
    for name, rel, kw in (("R", R, 0), ("S", S, 1)):
        p = str(tmp_path / f"{name}.rel")
        head = relfile.save(p, rel, kw, {"gen": "exp1", "nR": 4096, "nS": 20000, "theta": 0.8})
        rows, h2 = relfile.load(p)
        assert (np.asarray(rows) == rel).all()
        assert h2 == head and h2["key_word"] == kw
        assert head["checksum"] == relfile.checksum(rel)


def test_chunked_checksum_equals_whole():
    _, S = exp1_rels(1024, 10007)
    whole = relfile.checksum(S)
    parts = sum(relfile.checksum(S[a:a + 999], a) for a in range(0, len(S), 999)) & ((1 << 64) - 1)
    assert whole == parts
    T = S.copy()
    T[[3, 5]] = T[[5, 3]]  # row order matters
    assert relfile.checksum(T) != whole


def test_corruption_and_truncation_detected(tmp_path):
    R, _ = exp1_rels(2048, 4096)
    p = str(tmp_path / "R.rel")
    relfile.save(p, R)
    with open(p, "r+b") as f:
        f.seek(relfile.HEADER + 4 * 100)
        f.write(b"\x01\x02\x03\x04")
    with pytest.raises(ValueError, match="checksum"):
        relfile.load(p)
    with open(p, "r+b") as f:
        f.truncate(os.path.getsize(p) - 4)
    with pytest.raises(ValueError, match="truncated"):
        relfile.load(p)
    with open(p, "r+b") as f:
        f.write(b"XXXX")
    with pytest.raises(ValueError, match="not an hj3d relation"):
        relfile.read_header(p)


def test_cached_generates_once(tmp_path):
    p = str(tmp_path / "S.rel")
    calls = []

    def make():
        calls.append(1)
        return exp1_rels(1024, 8192)[1]

    meta = {"gen": "exp1", "nR": 1024, "nS": 8192, "theta": 0.8}
    a = relfile.cached(p, make, 1, meta)
    b = relfile.cached(p, make, 1, meta)
    assert len(calls) == 1 and (np.asarray(a) == np.asarray(b)).all()
    relfile.cached(p, make, 1, dict(meta, nS=8193 - 1, theta=1.0))  # other parameters: regenerated
    assert len(calls) == 2


@pytest.mark.gpu
def test_gpu_device_generated_relation_roundtrip(ctx, tmp_path):
    """A device-generated S (hj3d_gen_fk, the parallel non-parity generator) written to a file,
    mapped back and uploaded in chunks is the same relation, and joins the same."""
    import hj3d
    import torch
    nR, nS = 1 << 16, 1 << 20
    S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
    ctx.gen_keys(S, 0, 0, 0, 0)
    ctx.gen_fk(S, 1, 0, nR, 7)
    p = str(tmp_path / "S.rel")
    relfile.save(p, S.cpu().numpy().view(np.uint32), 1, {"gen": "device fk", "nR": nR, "seed": 7})
    rows, head = relfile.load(p)
    S2 = relfile.to_device(rows)
    assert torch.equal(S, S2) and head["n"] == nS
    R = torch.zeros((nR, 3), dtype=torch.int32, device="cuda")
    ctx.gen_keys(R, 0, 0, nR, 3)
    t = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, nR)
    t.build(hj3d.Rel(R, 0))
    a = ctx.probe(t, hj3d.Rel(S, 1), unique=True)
    b = ctx.probe(t, hj3d.Rel(S2, 1), unique=True)
    assert (a.n_out, a.n_cmps, a.sum_h, a.xor_h) == (b.n_out, b.n_cmps, b.sum_h, b.xor_h)
    t.close()
