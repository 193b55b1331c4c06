"""The N-rank HIP code path on ONE MI355X: world-size-2 runs of bench.py's multi-GPU path
(hj3d_partition bucket-range partitioner -> counts + pair all-to-all -> explicit-row build on the
owned bucket range -> chunked, accumulated probe), both ranks on cuda:0 with the gloo backend
staging the exchange through host memory (RCCL refuses two ranks on one device). The all-reduced
counters, output checksums and sharded-table statistics must equal the fixture the reference
binary wrote for the same relations (tests/golden/exp1_R1048576_S8388608_uni.json): the
verification step of bench.py compares them and the run fails otherwise.

The exchange as the product runs it: libhj3d's own RCCL communicator (hj3d_comm_*) at world size 1
(the box has one GPU): the partition -> count all-to-all -> asynchronous pair exchange (tickets) ->
build / chunked probe strand, its merge collectives, bench.py --dist-path, and the refusal of a
short receive buffer before the collective. tests/test_dropin.py runs the same strand from C++.

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


# ---- libhj3d's own RCCL exchange (hj3d_comm_*), world size 1 on the box's one GPU ----
STAT_KEYS = ("nb", "empty", "entries", "distinct", "cc0_min", "cc0_max", "cc0_sum", "cc0_cnt",
             "cc1_min", "cc1_max", "cc1_sum", "cc1_cnt")


@pytest.fixture(scope="module")
def comm(ctx):
    import hj3d
    c = hj3d.Comm(ctx, hj3d.Comm.unique_id(ctx), 0, 1)
    yield c
    c.close()


def test_runtime_is_single(ctx):
    """One HIP runtime mapped (torch's, shared by libhj3d.so): hj3d_ctx_create checks it."""
    import hj3d
    info = hj3d.runtime_info()
    assert "hip mapped=1" in info, info


@pytest.mark.parametrize("plan", ["Csr", "Nsr"])
def test_rccl_exchange_strand_equals_reference(ctx, comm, plan):
    """The multi-GPU strand of bench.py on libhj3d's communicator: hj3d_partition -> hj3d_comm_counts
    (3 probe chunks in one collective) -> hj3d_comm_exchange (asynchronous, on the exchange stream,
    tickets) -> explicit-row build / accumulated chunked probe, on the reference's relations
    (fixture exp1_R1048576_S8388608_uni): every counter, checksum and statistic equals the
    reference binary's. World size 1: RCCL sends each chunk to this rank itself."""
    import json
    import torch
    import hj3d
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "exp1_R1048576_S8388608_uni.json")))
    nR, nS = g["nR"], g["nS"]
    R, S = hj3d.exp1_relations_ref(nR, nS)
    nb = nR
    P, C = 1, 3
    unique, unnest = plan == "Csr", plan == "Nsr"
    kind = hj3d.HJ3D_CHAIN if plan == "Csr" else hj3d.HJ3D_NESTED
    dev = "cuda"
    # build side
    sendB = torch.empty((nR, 2), dtype=torch.int32, device=dev)
    cntB = torch.zeros((1, P), dtype=torch.int64, device=dev)
    ctx.partition(hj3d.Rel(R, 0), nb, P, sendB, cntB[0])
    scB, rcB = comm.counts(cntB)
    assert scB == [[nR]] and rcB == [[nR]]
    recvB = torch.empty((nR, 2), dtype=torch.int32, device=dev)
    rB, _ = comm.exchange(sendB, scB[0], rcB[0], recvB, asynchronous=False)
    t = hj3d.Table(ctx, kind, nb, *hj3d.part_range(nb, P, 0))
    t.build(hj3d.Rel(rB, key_word=0, row_word=1))
    # probe side in chunks, all counts in one collective, exchanges in flight together
    sb = [nS * c // C for c in range(C + 1)]
    sendP = torch.empty((nS, 2), dtype=torch.int32, device=dev)
    cntP = torch.zeros((C, P), dtype=torch.int64, device=dev)
    for c in range(C):
        ctx.partition(hj3d.Rel(S[sb[c]:sb[c + 1]], 1, row_base=sb[c]), nb, P, sendP[sb[c]:sb[c + 1]], cntP[c])
    scP, rcP = comm.counts(cntP)
    assert [r[0] for r in rcP] == [sb[c + 1] - sb[c] for c in range(C)]
    recvP = torch.empty((nS, 2), dtype=torch.int32, device=dev)
    pend, off = [], 0
    for c in range(C):
        v, tk = comm.exchange(sendP[sb[c]:sb[c + 1]], scP[c], rcP[c], recvP[off:])
        off += v.shape[0]
        pend.append((v, tk))
    for c, (v, tk) in enumerate(pend):
        comm.wait(tk)
        ctx.probe(t, hj3d.Rel(v, key_word=0, row_word=1), unique=unique, unnest=unnest, fetch=False,
                  accumulate=c > 0)
    r = ctx.probe_result()
    ref = g["plans"][plan]
    assert r.n_cmps == ref["c_cmp"]
    n_top = r.n_out
    assert n_top == ref["c_top"]
    got = {"n": r.n_out, "sum_a": r.sum_a, "sum_b": r.sum_b, "sum_h": r.sum_h, "xor_h": r.xor_h}
    assert got == {k: ref["out"][k] for k in got}
    # the counter merge of the multi-GPU verification (identity at world size 1)
    assert comm.allreduce_u64([r.n_cmps, 2**64 - 1]) == [r.n_cmps, 2**64 - 1]
    assert comm.allreduce_u64([7], hj3d.RED_MAX) == [7] and comm.allgather_u64(r.xor_h) == [r.xor_h]
    st = t.stats()
    assert {k: st[k] for k in STAT_KEYS} == {k: ref["stats"][k] for k in STAT_KEYS}
    t.close()


def test_rccl_exchange_short_buffer_is_refused(ctx, comm):
    """A receive buffer below the exchanged total is refused before the collective (HJ3D_EOVERFLOW)."""
    import torch
    import hj3d
    send = torch.zeros((100, 2), dtype=torch.int32, device="cuda")
    recv = torch.empty((99, 2), dtype=torch.int32, device="cuda")
    with pytest.raises(hj3d.Hj3dError) as e:
        comm.exchange(send, [100], [100], recv, asynchronous=False)
    assert e.value.status == hj3d.HJ3D_EOVERFLOW
    # the communicator is still usable
    v, _ = comm.exchange(send[:99], [99], [99], recv, asynchronous=False)
    assert v.shape[0] == 99


def test_rccl_counts_cap_refuses_before_the_exchange(ctx, comm):
    """hj3d_comm_counts_cap: with a receive capacity below the exchanged total the count exchange
    itself returns HJ3D_EOVERFLOW on every rank (agreed by an all-reduce), before any pair
    collective; tickets count up and an old ticket still orders the stream after its exchange."""
    import torch
    import hj3d
    from hj3d import dist as hdist
    counts = torch.tensor([[40], [60]], dtype=torch.int64, device="cuda")
    hdist.use_comm(comm)
    try:
        with pytest.raises(hdist.ExchangeOverflow):
            hdist.exchange_counts(counts, recv_cap=99)
        sc, rc = hdist.exchange_counts(counts, recv_cap=100)
        assert rc == [[40], [60]]
    finally:
        hdist.use_comm(None)
    send = torch.arange(200, dtype=torch.int32, device="cuda").view(100, 2)
    recv = torch.empty((100, 2), dtype=torch.int32, device="cuda")
    tickets = []
    for _ in range(70):  # more exchanges than ticket slots
        _, t = comm.exchange(send, [100], [100], recv, asynchronous=True)
        tickets.append(t)
    assert tickets == list(range(tickets[0], tickets[0] + 70))
    comm.wait(tickets[0])  # its slot was reused: waits for a later exchange of the same stream
    ctx.sync()
    assert torch.equal(recv, send)
    with pytest.raises(hj3d.Hj3dError):
        comm.wait(tickets[-1] + 1)  # never issued


@pytest.mark.parametrize("plan", ["Csr", "Nsr", "Nrs"])
def test_bench_dist_path_on_rccl_equals_reference(plan, tmp_path):
    """bench.py's multi-GPU strand with the exchange on libhj3d's RCCL communicator (--dist-path,
    world size 1): the verification step compares with the reference binary's fixture."""
    out = tmp_path / "line.json"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist-path", "--workload", "D",
           "--nR", "1048576", "--nS", "8388608", "--plan", plan, "--steps", "2", "--warmup", "1", "--chunks", "3",
           "--json-out", str(out), "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = json.loads(out.read_text())
    v = line["verification"]
    assert line["verified_bit_exact"], v
    assert "exp1_R1048576_S8388608_uni.json" in v["against"]
    assert line["config"]["exchange"].startswith("libhj3d")


def test_rccl_exchange_large_message(ctx, comm):
    """One chunk of more than 2^31 bytes (2^28 + 12345 pairs) arrives intact: the exchange moves
    8-byte words in pieces of at most 2^28 bytes, the library default (a 2e9-byte chunk of config D
    once came out corrupted as one message)."""
    import torch
    n = (1 << 28) + 12345
    send = torch.randint(-2**31, 2**31 - 1, (n, 2), dtype=torch.int32, device="cuda")
    recv = torch.empty_like(send)
    got, _ = comm.exchange(send, [n], [n], recv, asynchronous=False)
    ctx.sync()
    assert got.shape[0] == n and torch.equal(got, send)
    del send, recv, got
    torch.cuda.empty_cache()


def _exp4_fixture():
    import json
    return json.load(open(os.path.join(ROOT, "tests", "golden", "exp4_R16_a3_A4_b2_B2.json")))


def _exp4_check(plan, got, ref):
    for k in ("c_probe_RS", "c_probe_RS_cmp", "c_probe_RT", "c_probe_RT_cmp", "c_top"):
        assert got[k.lower()] == ref[k], (plan, k, got[k.lower()], ref[k])
    if plan == "Ndu":
        assert (got["c_unnest_1"], got["c_unnest_2"]) == (ref["c_unnest_1"], ref["c_unnest_2"])
    assert {k: got[k] for k in ("sum_a", "sum_b", "sum_c", "sum_h", "xor_h")} == \
           {k: ref["out"][k] for k in ("sum_a", "sum_b", "sum_c", "sum_h", "xor_h")}, plan


@pytest.mark.parametrize("plan", ["Ndu", "Chj"])
def test_rccl_exp4_strand_equals_reference(ctx, comm, plan):
    """Experiment 4 on the multi-GPU strand (hj3d.dist.exp4_join) with the exchange on libhj3d's RCCL
    communicator at world size 1: R, S, T co-partitioned, counts in one collective, three
    asynchronous pair exchanges, one hj3d_build_many, hj3d_probe2, counters all-reduced; equal to the
    reference binary's fixture exp4_R16_a3_A4_b2_B2."""
    import hj3d
    from hj3d import dist as hdist
    g = _exp4_fixture()
    R, S, T = hj3d.exp4_relations_ref(*g["generator_args"][1:6])
    hdist.use_comm(comm)  # (rank and world size from the communicator)
    try:
        got = hdist.exp4_join(ctx, plan, R, S, T, g["nb"])
    finally:
        hdist.use_comm(None)
    _exp4_check(plan, got, g["plans"][plan])


def _exp4_rank(rank, port, q):
    import torch
    import torch.distributed as dist
    import hj3d
    from hj3d import dist as hdist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        ctx = hj3d.Context(0)
        g = _exp4_fixture()
        R, S, T = hj3d.exp4_relations_ref(*g["generator_args"][1:6])
        sl = []
        for x in (R, S, T):
            lo, hi = rank * x.shape[0] // 2, (rank + 1) * x.shape[0] // 2
            sl.append((x[lo:hi].contiguous(), lo))
        out = {}
        for plan in ("Ndu", "Chj"):
            got = hdist.exp4_join(ctx, plan, sl[0][0], sl[1][0], sl[2][0], g["nb"], row_base=tuple(b for _, b in sl))
            out[plan] = {k: v for k, v in got.items()}
        torch.cuda.synchronize()
        ctx.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_exp4_two_rank_rehearsal_equals_reference():
    """hj3d.dist.exp4_join with two ranks on this one GPU (gloo, the exchange staged through host
    memory; RCCL allows one rank per device): each rank holds half of R, S and T, and both ranks'
    all-reduced results equal the reference binary's fixture."""
    import torch.multiprocessing as mp
    port = 29641  # (a fixed port, as the bench rehearsals above use: the RCCL communicator of this
    # process opens ephemeral sockets of its own)
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    procs = [mpc.Process(target=_exp4_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    g = _exp4_fixture()
    for plan in ("Ndu", "Chj"):
        assert res[0][plan]["per_rank"]["probe_tuples"] > 0 and res[1][plan]["per_rank"]["probe_tuples"] > 0
        for r in (0, 1):
            _exp4_check(plan, res[r][plan], g["plans"][plan])
