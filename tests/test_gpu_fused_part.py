"""GPU parity of the fused one-launch build partition (radix.hip k_rp_fused: histogram held in
registers, grid barrier, scatter) against the oracle, and against the two-launch form
(HJ3D_OPT_RP_UNFUSED) it replaces. Sizes cover every register-tile count the kernel is instantiated
for (1 to 6 tiles of 8192 tuples per workgroup), ragged last tiles and Zipf-skewed keys; the
chaining table's statistics, the unique and non-unique probes' counters and output checksums must
equal the oracle's (HtChaining1::insert order, ht_chaining.hh:181-196)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

STAT_KEYS = ("nb", "empty", "entries", "distinct", "cc0_min", "cc0_max", "cc0_sum", "cc0_cnt",
             "cc1_min", "cc1_max", "cc1_sum", "cc1_cnt")


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()


def _check(ctx, B, P, nb, unfused):
    import hj3d
    lib = hj3d.lib()
    ctx.rp_unfused(unfused)
    try:
        for unique in (True, False):
            e = O.chain_plan(B, 0, P, 1, nb, unique)
            t = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, nb)
            l0 = lib.hj3d_launch_count()
            t.build(hj3d.Rel(dev(B), 0))
            launches = lib.hj3d_launch_count() - l0
            r = ctx.probe(t, hj3d.Rel(dev(P), 1), unique=unique)
            assert (r.n_out, r.n_cmps) == (e.c_probe, e.c_cmp), (unique, unfused)
            assert {"n": r.n_out, "sum_a": r.sum_a, "sum_b": r.sum_b, "sum_c": 0, "sum_h": r.sum_h,
                    "xor_h": r.xor_h} == e.out, (unique, unfused)
            st = t.stats()
            assert {k: st[k] for k in STAT_KEYS} == {k: e.stats[k] for k in STAT_KEYS}, (unique, unfused)
            t.close()
    finally:
        ctx.rp_unfused(False)
    return launches


@pytest.mark.parametrize("n", [1_000_003, 2_500_017, 6_000_005, 9_437_184, 12_500_000])
@pytest.mark.parametrize("unfused", [False, True], ids=["fused", "two_launch"])
def test_fused_partition_chaining_build(ctx, n, unfused):
    """Key/FK tables at fill 1 (the headline's shape) from 1 to 6 tiles per workgroup; the fused
    form builds in two launches (partition + build), the two-launch form in three."""
    rng = np.random.default_rng(n % 1000)
    Bk = rng.permutation(n).astype(np.uint32)
    Pk = rng.integers(0, n, n // 2).astype(np.uint32)
    B = O.tuples3(Bk, np.zeros(n, np.uint32))
    P = O.tuples3(np.arange(len(Pk), dtype=np.uint32), Pk)
    launches = _check(ctx, B, P, n, unfused)
    assert launches == (3 if unfused else 2), launches


@pytest.mark.parametrize("theta", [0.6, 1.0])
def test_fused_partition_skewed_keys(ctx, theta):
    """Zipf build keys: hot buckets make partitions of very different sizes (one exceeds the staged
    build's registers and takes its HBM fallback); the fused partition's runs stay exact."""
    rng = np.random.default_rng(int(theta * 100))
    n = 4_000_000
    Bk = (np.minimum(rng.zipf(1.0 + theta, n), 5_000_000) - 1).astype(np.uint32)
    Pk = rng.integers(0, 4_000_000, n).astype(np.uint32)
    B = O.tuples3(Bk, np.zeros(n, np.uint32))
    P = O.tuples3(np.arange(n, dtype=np.uint32), Pk)
    assert _check(ctx, B, P, n, False) == 2


def test_fused_partition_repeated_builds(ctx):
    """The grid barrier's arrival counter is monotonic across launches (never reset): many builds
    on one context, alternating table sizes (grids of 122 and 256 workgroups), stay exact."""
    import hj3d
    rng = np.random.default_rng(5)
    for k in range(12):
        n = 1_000_000 if k % 2 else 3_000_000
        Bk = rng.permutation(n).astype(np.uint32)
        B = O.tuples3(Bk, np.zeros(n, np.uint32))
        P = O.tuples3(np.arange(n // 4, dtype=np.uint32), rng.integers(0, n, n // 4).astype(np.uint32))
        e = O.chain_plan(B, 0, P, 1, n, True)
        t = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, n)
        t.build(hj3d.Rel(dev(B), 0))
        r = ctx.probe(t, hj3d.Rel(dev(P), 1), unique=True)
        assert (r.n_out, r.n_cmps, r.sum_h, r.xor_h) == (e.c_probe, e.c_cmp, e.out["sum_h"], e.out["xor_h"]), k
        t.close()


def test_timing_events_measure_the_stream(ctx):
    """hj3d_tevent_* (fence-free HIP events on the context stream, the bench's phase boundaries):
    the span around a build equals the span torch.cuda.Event measures around the same work within
    the events' jitter, and spans are ordered."""
    import torch
    import hj3d
    n = 4_000_000
    B = O.tuples3(np.random.default_rng(3).permutation(n).astype(np.uint32), np.zeros(n, np.uint32))
    dB = dev(B)
    t = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, n)
    t.build(hj3d.Rel(dB, 0))
    torch.cuda.synchronize()
    ev = [hj3d.TimingEvent(ctx) for _ in range(3)]
    te = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    te[0].record()
    ev[0].record()
    for _ in range(5):
        t.build(hj3d.Rel(dB, 0))
    ev[1].record()
    t.build(hj3d.Rel(dB, 0))
    ev[2].record()
    te[1].record()
    torch.cuda.synchronize()
    a, b = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
    total = te[0].elapsed_time(te[1])
    assert 0 < b < a and a + b <= total * 1.05 + 0.05, (a, b, total)
    assert a + b >= 0.5 * total, (a, b, total)
    t.close()


def test_fused_partition_barrier_timeout_is_reported(ctx):
    """The fused partition's failure path (HJ3D_OPT_DIAG_GBAR: its grid barrier cannot complete, every
    workgroup times out after 1 ms and goes on with partial sizes): the table's statistics, size,
    export and finish, and the next probe result, return HJ3D_EDEVICE; the context's arrival counter
    stays in step, so the next build on the same context is exact again and reads clean."""
    import hj3d
    rng = np.random.default_rng(11)
    n = 3_000_000
    B = O.tuples3(rng.permutation(n).astype(np.uint32), np.zeros(n, np.uint32))
    P = O.tuples3(np.arange(n // 2, dtype=np.uint32), rng.integers(0, n, n // 2).astype(np.uint32))
    e = O.chain_plan(B, 0, P, 1, n, True)
    dB, dP = dev(B), dev(P)
    t = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, n)
    ctx.diag_gbar(100_000)  # 1 ms
    try:
        t.build(hj3d.Rel(dB, 0))
    finally:
        ctx.diag_gbar(0)
    assert t.build_path(finish=False) == "radix", t.build_path(finish=False)
    import ctypes as C
    lib = hj3d.lib()
    npay, nsub = C.c_uint64(), C.c_uint64()
    for what, call in (("stats", t.stats), ("finish", t.finish),
                       ("size", lambda: ctx._check(lib.hj3d_table_size(ctx.h, t.h, None, None), "size")),
                       ("export", lambda: ctx._check(lib.hj3d_table_export(ctx.h, t.h, None, None, None, C.byref(npay),
                                                                           C.byref(nsub)), "export"))):
        with pytest.raises(hj3d.Hj3dError) as ei:
            call()
        assert ei.value.status == hj3d.HJ3D_EDEVICE, what
        assert "barrier" in str(ei.value), what
    with pytest.raises(hj3d.Hj3dError) as ei:
        ctx.probe(t, hj3d.Rel(dP, 1), unique=True)
    assert ei.value.status == hj3d.HJ3D_EDEVICE
    # a rebuild on the same context (and the same table) is exact and reads clean
    for _ in range(3):
        t.build(hj3d.Rel(dB, 0))
        r = ctx.probe(t, hj3d.Rel(dP, 1), unique=True)
        assert (r.n_out, r.n_cmps, r.sum_h, r.xor_h) == (e.c_probe, e.c_cmp, e.out["sum_h"], e.out["xor_h"])
        st = t.stats()
        assert {k: st[k] for k in STAT_KEYS} == {k: e.stats[k] for k in STAT_KEYS}
    t.close()
