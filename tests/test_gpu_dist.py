"""The N-rank HIP code path on ONE MI355X: world-size-2 runs of bench.py's multi-GPU path
(hj3d_partition bucket-range partitioner -> counts + pair all-to-all -> explicit-row build on the
owned bucket range -> chunked, accumulated probe), both ranks on cuda:0 with the gloo backend
staging the exchange through host memory (RCCL refuses two ranks on one device). The all-reduced
counters, output checksums and sharded-table statistics must equal the fixture the reference
binary wrote for the same relations (tests/golden/exp1_R1048576_S8388608_uni.json): the
verification step of bench.py compares them and the run fails otherwise.

Also: output overflow of an accumulated, non-dense probe strand is reported (HJ3D_EOVERFLOW)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("plan", ["Csr", "Nsr", "Nrs"])
def test_two_rank_partitioned_join_equals_reference(plan, tmp_path):
    out = tmp_path / "line.json"
    port = 29611 + ["Csr", "Nsr", "Nrs"].index(plan)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--rehearse", "--workload", "D", "--nR", "1048576", "--nS", "8388608", "--plan", plan,
           "--steps", "2", "--warmup", "1", "--chunks", "3", "--json-out", str(out)]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = json.loads(out.read_text())
    v = line["verification"]
    assert line["verified_bit_exact"], v
    assert "exp1_R1048576_S8388608_uni.json" in v["against"]
    assert v["out"] and v["c_htProbeCmp"] and v["c_top"] and v["stats"], v
    assert line["n_gpus"] == 2 and line["per_gpu"]["probe_tuples"]["min"] > 0


def test_accumulated_unnest_overflow_is_reported(ctx):
    """HJ3D_PROBE_ACCUMULATE with a non-dense (unnest) output: a chunk whose output exceeds its own
    buffer makes hj3d_probe_result report HJ3D_EOVERFLOW, even though earlier chunks fit."""
    import numpy as np
    import torch
    import hj3d
    nR, nS = 4096, 65536
    rng = np.random.default_rng(3)
    Rk = rng.permutation(nR).astype(np.uint32)
    Sa = rng.integers(0, nR, nS).astype(np.uint32)
    R = torch.zeros((nR, 3), dtype=torch.int32, device="cuda")
    S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
    R[:, 0] = torch.from_numpy(Rk.view(np.int32)).cuda()
    S[:, 0] = torch.arange(nS, dtype=torch.int32, device="cuda")
    S[:, 1] = torch.from_numpy(Sa.view(np.int32)).cuda()
    t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nR)
    t.build(hj3d.Rel(R, 0))
    half = nS // 2
    big = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    # both chunks fit: no overflow, counters of the whole strand
    ctx.probe(t, hj3d.Rel(S[:half], 1), unnest=True, out=big[:half], fetch=False)
    ctx.probe(t, hj3d.Rel(S[half:], 1, row_base=half), unnest=True, out=big[half:], fetch=False, accumulate=True)
    r = ctx.probe_result()
    assert not r.overflow and r.n_out == nS
    # the second chunk gets a buffer one pair short
    ctx.probe(t, hj3d.Rel(S[:half], 1), unnest=True, out=big[:half], fetch=False)
    ctx.probe(t, hj3d.Rel(S[half:], 1, row_base=half), unnest=True, out=big[half:nS - 1], fetch=False,
              accumulate=True)
    r = ctx.probe_result()
    assert r.overflow and r.n_out == nS
    # a later chunk that fits does not clear the strand's overflow
    ctx.probe(t, hj3d.Rel(S[:16], 1), unnest=True, out=big[:16], fetch=False, accumulate=True)
    assert ctx.probe_result().overflow
    # a new strand starts clean
    ctx.probe(t, hj3d.Rel(S, 1), unnest=True, out=big, fetch=False)
    assert not ctx.probe_result().overflow
