"""#dv pre-pass (hj3d_key_bitmap) on its tiled path: the bitmap must equal the set of keys below the
domain bit for bit, and the outside count the keys at or above it — for every relation layout the
partition pass reads (12-B tuples with the key in word 0, 1 or 2 through 16-B loads; unaligned bases,
8-B pairs through the generic load), slice counts from 1 to 1024, ragged tiles and Zipf skew. The
distinct count itself is pinned against the reference's numDvSa in test_gpu_parity.py and, at config
C size, test_gpu_headline.py (main_experiment1.cc:453-454)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def ref_bitmap(keys: np.ndarray, domain: int) -> tuple[np.ndarray, int]:
    words = (domain + 31) // 32
    k = keys[keys.astype(np.uint64) < domain].astype(np.int64)
    bits = np.zeros(words * 32, dtype=bool)
    bits[k] = True
    bm = np.packbits(bits.reshape(-1, 8), axis=1, bitorder="little").reshape(-1).view(np.uint32)
    return bm, int((keys.astype(np.uint64) >= domain).sum())


def run(ctx, tensor, key_word, domain, prefill=None):
    import torch
    import hj3d
    words = (domain + 31) // 32
    bm = torch.zeros(words, dtype=torch.int32, device="cuda")
    if prefill is not None:
        bm.copy_(torch.from_numpy(prefill.view(np.int32)))
    out = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.key_bitmap(hj3d.Rel(tensor, key_word=key_word), domain, bm, out)
    return bm.cpu().numpy().view(np.uint32), int(out.item())


CASES = [  # (n, words per tuple, key word, domain, zipf theta or 0)
    (1 << 20, 3, 1, 10_000_000, 0.0),          # config C shape: 16 slices
    (3_000_017, 3, 0, 1 << 20, 0.8),           # ragged last tile, Zipf, 2 slices
    (2_000_003, 3, 2, 5_000, 0.0),             # one slice (157 words), most keys outside
    (1_500_000, 2, 0, 100_000_000, 0.0),       # 8-B pairs: generic loads, 256 slices
    (1_200_000, 3, 1, (1 << 32) // 7, 1.0),    # 1024 slices, heavy skew
]


@pytest.mark.parametrize("n,w,kw,domain,theta", CASES)
def test_key_bitmap_tiled_exact(ctx, n, w, kw, domain, theta):
    import torch
    rng = np.random.default_rng(n + kw)
    hi = min(domain + domain // 8 + 1, 1 << 32)
    if theta:
        keys = ((rng.zipf(1.0 + theta, n) * 2654435761) % hi).astype(np.uint32)
    else:
        keys = rng.integers(0, hi, n, dtype=np.uint64).astype(np.uint32)
    t = rng.integers(0, 1 << 31, (n, w), dtype=np.int64).astype(np.int32)
    t[:, kw] = keys.view(np.int32)
    got, nout = run(ctx, torch.from_numpy(t).cuda(), kw, domain)
    exp, eout = ref_bitmap(keys, domain)
    assert nout == eout
    assert np.array_equal(got, exp)


def test_key_bitmap_tiled_unaligned_and_or_into(ctx):
    """A relation whose base is not 16-B aligned (rows from 1) takes the generic load; the call ORs
    into a bitmap that already holds bits (the multi-GPU rows and repeated calls rely on it)."""
    import torch
    rng = np.random.default_rng(7)
    n, domain = 1_300_001, 3_000_000
    t = rng.integers(0, domain, (n + 1, 3), dtype=np.int64).astype(np.int32)
    dt = torch.from_numpy(t).cuda()
    pre = np.zeros((domain + 31) // 32, dtype=np.uint32)
    pre[::5] = 0x80000001
    got, nout = run(ctx, dt[1:], 2, domain, prefill=pre)
    exp, _ = ref_bitmap(t[1:, 2].view(np.uint32), domain)
    assert nout == 0
    assert np.array_equal(got, exp | pre)
