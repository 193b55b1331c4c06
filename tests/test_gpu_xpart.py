"""GPU parity of the single-pass exchange partitioner (hj3d_partition_strided): per
destination, the same (key, row) pairs as the stable two-pass hj3d_partition (compared as sorted
sets: the single pass keeps no order inside a destination), at the strided layout the exchange
sends from; empty, one-tuple and ragged inputs, 1 to 256 destinations, skewed keys, explicit rows,
a selection below the exchange. The counters of a bucket-range split probed from the single-pass
output equal the golden fixture (test_gpu_parity.py's shard test) and, at config D's size, the
reference binary's (test_gpu_headline.py, 8-owner split)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to("cuda")


def _fmix32(x):
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(13)
    x = (x * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    return x


def _sorted_rows(a):
    a = np.asarray(a, dtype=np.uint32).reshape(-1, 2)
    return a[np.lexsort((a[:, 1], a[:, 0]))]


def _compare(ctx, rel, n, nb, parts, preds=None, stride=None):
    import torch
    stable = torch.empty((max(n, 1), 2), dtype=torch.int32, device="cuda")
    cs = torch.zeros(parts, dtype=torch.int64, device="cuda")
    ctx.partition(rel, nb, parts, stable, cs, preds=preds)
    stride = max(n, 1) if stride is None else stride
    single = torch.full((max(parts * stride, 1), 2), -1, dtype=torch.int32, device="cuda")
    cx = torch.full((parts,), 12345, dtype=torch.int64, device="cuda")  # the call zeroes its counts
    ctx.partition(rel, nb, parts, single, cx, preds=preds, stride=stride)
    a, b = cs.cpu().tolist(), cx.cpu().tolist()
    assert a == b
    st = stable.cpu().numpy().view(np.uint32)
    sg = single.cpu().numpy().view(np.uint32)
    off = 0
    for p in range(parts):
        exp = st[off:off + a[p]]
        w = min(a[p], stride)
        got = sg[p * stride:p * stride + w]
        if w == a[p]:
            assert (_sorted_rows(got) == _sorted_rows(exp)).all(), p
        else:  # spilled: the area holds `stride` of the destination's pairs, each exactly once
            e = {tuple(x) for x in _sorted_rows(exp).tolist()}
            g = [tuple(x) for x in _sorted_rows(got).tolist()]
            assert len(set(g)) == len(g) == stride and set(g) <= e, p
        # nothing past the destination's count was written
        if a[p] < stride:
            assert (sg[p * stride + a[p]:(p + 1) * stride] == 0xFFFFFFFF).all(), p
        off += a[p]
    return a


@pytest.mark.parametrize("parts", [1, 3, 8, 256])
@pytest.mark.parametrize("n", [0, 1, 8191, 8192, 8193, 1_000_003])
def test_single_pass_matches_stable(ctx, parts, n):
    import hj3d
    rng = np.random.default_rng(n + parts)
    nb = 100_003
    t = np.stack([np.arange(n, dtype=np.uint32), rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
                  np.zeros(n, dtype=np.uint32)], axis=1)
    base = t if n else np.zeros((1, 3), dtype=np.uint32)  # n = 0: a one-row tensor, no tuple in it
    counts = _compare(ctx, hj3d.Rel(dev(base), key_word=1, n=n), n, nb, parts)
    assert sum(counts) == n


@pytest.mark.parametrize("parts", [2, 8])
def test_single_pass_skewed_explicit_rows(ctx, parts):
    """Zipf keys (one destination takes most tuples) with explicit row ids (received pairs)."""
    import hj3d
    _, Sa, _ = O.gen_exp1(1 << 16, 2_000_000, True, 1.0, 0)
    rng = np.random.default_rng(5)
    rows = rng.permutation(len(Sa)).astype(np.uint32)
    t = np.stack([Sa, rows], axis=1).astype(np.uint32)
    counts = _compare(ctx, hj3d.Rel(dev(t), key_word=0, row_word=1), len(t), 1 << 16, parts)
    assert max(counts) - min(counts) > len(t) // 20  # the hot keys' destination stands out


@pytest.mark.parametrize("parts", [3, 8])
def test_single_pass_with_selection(ctx, parts):
    import hj3d
    n, nb = 300_001, 100_003
    rng = np.random.default_rng(11)
    t = np.stack([rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
                  rng.integers(0, nb, n).astype(np.uint32),
                  rng.integers(0, 100, n).astype(np.uint32)], axis=1)
    preds = [(2, ">=", 25), (2, "<", 75)]
    counts = _compare(ctx, hj3d.Rel(dev(t), 1), n, nb, parts, preds=preds)
    sel = O.select(t, 1, preds)
    owner = ((_fmix32(sel[:, 0]) % np.uint64(nb)) * np.uint64(parts) // np.uint64(nb)).astype(np.int64)
    assert counts == [int((owner == d).sum()) for d in range(parts)]


@pytest.mark.parametrize("parts", [2, 8, 64])
def test_single_pass_bounded_stride(ctx, parts):
    """The library's bounded stride (hj3d_partition_stride: mean + 8 sigma + 2 tiles) holds every
    destination of distinct keys: no spill, parts x stride pairs of send buffer instead of parts x n."""
    import hj3d
    n, nb = 4_000_037, 3_999_971
    rng = np.random.default_rng(parts)
    t = np.stack([rng.permutation(n).astype(np.uint32), np.arange(n, dtype=np.uint32)], axis=1)
    stride = hj3d.partition_stride(n, parts)
    assert stride < n and parts * stride < 1.02 * n + parts * 40_000
    counts = _compare(ctx, hj3d.Rel(dev(t), key_word=0, row_word=1), n, nb, parts, stride=stride)
    assert max(counts) <= stride and sum(counts) == n


def test_single_pass_spill_reported_by_counts(ctx):
    """A destination above its stride spills: its count still counts every tuple, exactly `stride`
    of its pairs are written, nothing outside the areas (the caller then re-partitions)."""
    import hj3d
    _, Sa, _ = O.gen_exp1(1 << 16, 400_000, True, 1.0, 0)
    t = np.stack([Sa, np.arange(len(Sa), dtype=np.uint32)], axis=1).astype(np.uint32)
    stride = hj3d.partition_stride(len(t), 4)
    counts = _compare(ctx, hj3d.Rel(dev(t), key_word=0, row_word=1), len(t), 1 << 16, 4, stride=stride)
    assert max(counts) > stride and sum(counts) == len(t)


def test_single_pass_refuses_zero_stride(ctx):
    import torch
    import hj3d
    t = np.zeros((100, 3), dtype=np.uint32)
    out = torch.empty((800, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    with pytest.raises(hj3d.Hj3dError):
        ctx.partition(hj3d.Rel(dev(t), 1), 1000, 8, out, cnt, stride=0)
