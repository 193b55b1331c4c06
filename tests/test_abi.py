"""The C-ABI library: it loads, exports every function include/hj3d.h declares, and its
host-only helpers agree with the Python definitions. No device compute here (CPU suite)."""
import ctypes as C

import pytest

import hj3d


def test_library_exports_every_declared_symbol():
    L = hj3d.lib()
    declared = hj3d.declared_symbols()
    assert len(declared) >= 20
    missing = [s for s in declared if not hasattr(L, s)]
    assert missing == []


def test_mix64_definition_shared_with_oracle():
    import oracle as O
    for z in (0, 1, 0xdeadbeef, (7 << 32) | 3, (1 << 64) - 1):
        assert hj3d.lib().hj3d_mix64(z) == hj3d.mix64(z) == O.mix64(z)


@pytest.mark.parametrize("nb,parts", [(1, 1), (1, 8), (7, 8), (10_000_000, 8), (1_000_003, 3), (4_000_000_000, 5)])
def test_part_range_matches_owner_function(nb, parts):
    # owner(b) = b * parts // nb (part.hip); the ranges must tile [0, nb) exactly
    prev = 0
    for p in range(parts):
        lo, hi = hj3d.part_range(nb, parts, p)
        assert lo == prev and lo <= hi
        for b in {lo, hi - 1} if hi > lo else set():
            assert b * parts // nb == p
        prev = hi
    assert prev == nb


def test_context_fails_loudly_without_device():
    """No silent CPU fallback: without a GPU the engine refuses to create a context."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = C.c_void_p()
    assert hj3d.lib().hj3d_ctx_create(0, None, C.byref(h)) == hj3d.HJ3D_EDEVICE
    with pytest.raises(RuntimeError):
        hj3d.Context(0)


def test_null_and_invalid_arguments_rejected():
    L = hj3d.lib()
    assert L.hj3d_ctx_create(0, None, None) == hj3d.HJ3D_EINVAL
    assert L.hj3d_build(None, None, None) == hj3d.HJ3D_EINVAL
    assert L.hj3d_probe(None, None, None, 0, None, 0) == hj3d.HJ3D_EINVAL
    assert L.hj3d_table_create(None, None, None) == hj3d.HJ3D_EINVAL


def test_single_hip_runtime_mapped():
    """The loader maps torch first, so libhj3d.so binds torch's HIP runtime: exactly one libamdhip64
    in the process (hj3d_ctx_create refuses to run with two). No GPU needed."""
    import hj3d
    info = hj3d.runtime_info()
    assert "hip mapped=1" in info, info
    assert "libamdhip64" in info, info


@pytest.mark.parametrize("n,parts", [(0, 8), (1, 8), (1000, 8), (25_000_000, 8), (250_000_000, 8), (10**9, 2),
                                     (10**8, 256), (12345, 1)])
def test_partition_stride_bounds(n, parts):
    """hj3d_partition_stride (host-only): at least the mean destination count plus 8 sigma (distinct
    keys spill with negligible probability), at most n (stride n never spills), and for large
    inputs about n / parts, so parts x stride pairs of send buffer stay near n."""
    import math
    s = hj3d.partition_stride(n, parts)
    assert s <= n
    if parts == 1:
        assert s == n
        return
    m = n / parts
    assert s >= min(n, m + max(8 * math.sqrt(m * (1 - 1 / parts)), m / 64))
    if n >= 10**7:
        assert parts * s < 1.02 * n + parts * 20_000


def test_table_build_path_before_build():
    """hj3d_table_build_path is "none" for a null or unbuilt table (no device needed)."""
    assert hj3d.lib().hj3d_table_build_path(None) == b"none"
