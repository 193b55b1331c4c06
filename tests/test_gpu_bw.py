"""The same-run streaming-copy peak (hj3d_stream_copy) that every bench line carries:
the copy is a real copy (destination equals source, ragged sizes included) and its rate is a
plausible HBM rate (between 1 TB/s and the 8 TB/s spec)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbytes", [16, 4096 + 16, 256 << 20])
def test_stream_copy_copies_and_reports_a_rate(ctx, nbytes):
    import torch
    src = torch.randint(-2**31, 2**31 - 1, (nbytes // 4,), dtype=torch.int32, device="cuda")
    dst = torch.zeros_like(src)
    r = ctx.stream_copy_peak(dst, src, 3)
    torch.cuda.synchronize()
    assert torch.equal(dst, src)
    assert r["bytes_copied"] == nbytes and r["copy_peak_GBs"] >= r["copy_median_GBs"] > 0
    if nbytes >= (256 << 20):
        assert 1000.0 < r["copy_peak_GBs"] < 8000.0, r
