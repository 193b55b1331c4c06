"""Multi-GPU path rehearsed on CPU: world size 2, gloo backend.

Each rank holds a contiguous slice of R and S (global row ids), partitions it by bucket range
exactly as hj3d_partition does (owner = bucket * P / NB, stable; restated here in numpy; the probe
side as hj3d_partition_strided lays it out: strided, no order inside an owner),
exchanges (key, row) pairs with hj3d.dist.exchange (all_to_all; the probe side in chunks through
exchange_counts + exchange_pairs_async as bench.py does), and joins its received pairs
with the oracle over the full bucket space (only its own buckets are populated). The per-rank
counters, all-reduced with hj3d.dist, must equal the single-table oracle on the whole relations:
join cardinality, c_htProbeCmp, unnest counts, output checksums and the table statistics.
#dv(S.a), which sizes the build-on-S.a plans, comes from the distributed pre-pass
(hj3d.dist.num_distinct: bitmap slices all-to-all'ed, OR + popcount, summed).
That is the property the device path relies on (bucket ranges keep per-bucket chain order when
received segments are concatenated in source-rank order)."""
import os
import socket

import numpy as np
import pytest

import oracle as O

WORLD = 2


def murmur32(x):
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x = (x * np.uint32(0x85EBCA6B)).astype(np.uint32)
    x ^= x >> np.uint32(13)
    x = (x * np.uint32(0xC2B2AE35)).astype(np.uint32)
    x ^= x >> np.uint32(16)
    return x


def partition(keys, rows, nb, parts):
    """(key, row) pairs grouped by owner(bucket) = bucket * parts // nb, stable (hj3d_partition)."""
    b = (murmur32(keys).astype(np.uint64) % np.uint64(nb)).astype(np.uint64)
    owner = (b * np.uint64(parts) // np.uint64(nb)).astype(np.int64)
    order = np.argsort(owner, kind="stable")
    pairs = np.stack([keys[order], rows[order]], axis=1).astype(np.uint32)
    counts = np.bincount(owner, minlength=parts).astype(np.int64)
    return pairs, counts


def partition_strided(keys, rows, nb, parts, seed):
    """hj3d_partition_strided's layout: owner p's pairs at rows [p * n, p * n + counts[p]) of a
    (parts * n, 2) buffer, in NO particular order inside an owner (shuffled here; the device's
    order depends on run claims), the rest of each area garbage."""
    n = len(keys)
    pairs, counts = partition(keys, rows, nb, parts)
    out = np.full((max(parts * n, 1), 2), 0xDEADBEEF, dtype=np.uint32)
    rng = np.random.default_rng(seed)
    starts = np.concatenate([[0], np.cumsum(counts)])
    for p in range(parts):
        blk = pairs[starts[p]:starts[p + 1]]
        out[p * n:p * n + counts[p]] = blk[rng.permutation(len(blk))]
    return out, counts


def bitmap_np(keys, words):
    """Bit k set for every key k (hj3d_key_bitmap restated)."""
    bm = np.zeros(words, dtype=np.uint32)
    np.bitwise_or.at(bm, keys >> 5, np.left_shift(np.uint32(1), (keys & 31).astype(np.uint32)))
    return bm


def or_popcount_np(slices):
    """popcount of the OR over the rows (hj3d_bitmap_or_popcount restated)."""
    x = np.bitwise_or.reduce(slices.numpy().view(np.uint32), axis=0)
    return int(np.unpackbits(x.view(np.uint8)).sum())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, case, q):
    import torch
    import torch.distributed as dist
    import hj3d
    from hj3d import dist as hdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        nR, nS, skew = case
        Rk, Sa, _ = O.gen_exp1(nR, nS, skew, 1.0, 0)
        # the #dv pre-pass: bitmaps of the local S.a slices, all-to-all'ed slices, OR + popcount
        lo_s, hi_s = rank * nS // WORLD, (rank + 1) * nS // WORLD
        words = -(-nR // 32)
        words = -(-words // WORLD) * WORLD
        bm = bitmap_np(Sa[lo_s:hi_s], words)
        dv = hdist.num_distinct(torch.from_numpy(bm.view(np.int32)), or_popcount_np)
        assert dv == O.num_distinct(Sa)
        out = {}
        for plan, (bkeys, pkeys, nb) in {
            "Csr": (Rk, Sa, nR), "Nsr": (Rk, Sa, nR), "Crs": (Sa, Rk, dv), "Nrs": (Sa, Rk, dv),
        }.items():
            # contiguous slices of the build and probe relations, global row ids
            def local(keys):
                n = len(keys)
                lo, hi = rank * n // WORLD, (rank + 1) * n // WORLD
                return keys[lo:hi], np.arange(lo, hi, dtype=np.uint32)

            recv = []
            k, r = local(bkeys)
            pairs, counts = partition(k, r, nb, WORLD)
            got = hdist.exchange(torch.from_numpy(pairs.view(np.int32)), torch.from_numpy(counts))
            recv.append(got.numpy().view(np.uint32))
            # the probe side as bench.py ships it: 3 chunks partitioned separately (the single-pass
            # partitioner's strided, unordered layout), all chunks' counts in one collective, then one
            # pair all-to-all per chunk into one receive buffer
            k, r = local(pkeys)
            cb = [len(k) * c // 3 for c in range(4)]
            parts = [partition_strided(k[cb[c]:cb[c + 1]], r[cb[c]:cb[c + 1]], nb, WORLD, seed=rank * 3 + c)
                     for c in range(3)]
            sc, rc = hdist.exchange_counts(torch.from_numpy(np.stack([pc for _, pc in parts])))
            assert sc == [pc.tolist() for _, pc in parts]
            rbuf = torch.empty((sum(map(sum, rc)), 2), dtype=torch.int32)
            off = 0
            for c in range(3):
                got, work = hdist.exchange_pairs_async(torch.from_numpy(parts[c][0].view(np.int32)), sc[c], rc[c],
                                                       rbuf[off:], send_stride=cb[c + 1] - cb[c])
                assert work is None or work.wait()
                off += got.shape[0]
            recv.append(rbuf.numpy().view(np.uint32))
            # the owned bucket range agrees with hj3d_part_range
            lo, hi = hj3d.part_range(nb, WORLD, rank)
            bk = murmur32(recv[0][:, 0]).astype(np.uint64) % np.uint64(nb)
            assert ((bk >= lo) & (bk < hi)).all()
            if plan.startswith("C"):
                e = O.chain_plan(recv[0], 0, recv[1], 0, nb, plan == "Csr", brow=1, prow=1)
            else:
                e = O.nested_plan(recv[0], 0, recv[1], 0, nb, True, brow=1, prow=1)
            st = e.stats
            owned = hi - lo
            sums = [e.c_probe, e.c_cmp, e.c_unnest, e.c_top, e.out["n"], e.out["sum_a"], e.out["sum_b"],
                    e.out["sum_h"], st["empty"] - (nb - owned), st["entries"], st["distinct"], st["cc0_sum"],
                    st["cc1_sum"], st["cc1_cnt"]]
            tot = hdist.allreduce_sum_u64(sums, "cpu")
            x = hdist.allreduce_xor_u64(e.out["xor_h"], "cpu")
            mx = hdist.allreduce_max(float(st["cc0_max"]), "cpu")
            # the statistics of this rank's shard (its owned bucket range), reduced as bench.py does
            shard = dict(st, nb=owned, empty=st["empty"] - (nb - owned), cc0_cnt=owned, cc0_min=0)
            red = hdist.allreduce_stats(shard, "cpu")
            out[plan] = (tot, x, int(mx), red)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", [(4096, 32768, False), (2048, 65536, True)], ids=["uniform", "zipf"])
def test_bucket_range_exchange_world2(case):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, case, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nR, nS, skew = case
    Rk, Sa, _ = O.gen_exp1(nR, nS, skew, 1.0, 0)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    dv = O.num_distinct(Sa)
    exp = {"Csr": O.chain_plan(R, 0, S, 1, nR, True), "Nsr": O.nested_plan(R, 0, S, 1, nR, True),
           "Crs": O.chain_plan(S, 1, R, 0, dv, False), "Nrs": O.nested_plan(S, 1, R, 0, dv, True)}
    for plan, e in exp.items():
        tot, x, mx, red = res[0][plan]
        assert res[1][plan] == res[0][plan]  # every rank sees the same reduced values
        st = e.stats
        want = [e.c_probe, e.c_cmp, e.c_unnest, e.c_top, e.out["n"], e.out["sum_a"], e.out["sum_b"], e.out["sum_h"],
                st["empty"], st["entries"], st["distinct"], st["cc0_sum"], st["cc1_sum"], st["cc1_cnt"]]
        assert tot == [v & ((1 << 64) - 1) for v in want], plan
        assert x == e.out["xor_h"] and mx == st["cc0_max"], plan
        for k in ("nb", "empty", "entries", "distinct", "cc0_sum", "cc0_cnt", "cc1_sum", "cc1_cnt", "cc0_max",
                  "cc1_max", "cc1_min"):
            assert red[k] == st[k], (plan, k, red[k], st[k])


def _short_worker(rank, port, q):
    import torch
    import torch.distributed as dist
    from hj3d import dist as hdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        # every rank sends 10 pairs to each peer; rank 1's receive buffer holds only 15
        counts = torch.full((2, WORLD), 5, dtype=torch.int64)
        cap = 15 if rank == 1 else 20
        outcome = "ok"
        try:
            hdist.exchange_counts(counts, recv_cap=cap)
        except hdist.ExchangeOverflow as e:
            outcome = "short" if "arrive at this rank" in str(e) else "peer short"
        # the process group is still usable: a full-size exchange afterwards goes through
        sc, rc = hdist.exchange_counts(counts, recv_cap=20)
        q.put((rank, outcome, sum(map(sum, rc))))
    finally:
        dist.destroy_process_group()


def test_exchange_refusal_is_collective():
    """ADVICE / VERDICT r2: a short receive buffer on ONE rank makes EVERY rank refuse the exchange
    before any pair collective (exchange_counts with recv_cap: the ranks agree by one all-reduce),
    instead of the short rank refusing alone and its peers waiting in the pair all-to-all."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_short_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {r: (o, n) for r, o, n in (q.get(timeout=120) for _ in range(WORLD))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: ("peer short", 20), 1: ("short", 20)}


EXP4_KEYS = ("c_probe_rs", "c_probe_rs_cmp", "c_probe_rt", "c_probe_rt_cmp", "c_unnest_1", "c_unnest_2", "c_top")


def _exp4_worker(rank, port, q):
    """Experiment 4 on the multi-GPU strand's layout (hj3d.dist.exp4_join's steps, the join done by the
    oracle): R, S, T co-partitioned by bucket range of the one FK hash, all counts in one collective,
    three pair all-to-alls, the rank's Ndu / Chj over its received pairs, counters all-reduced."""
    import json
    import torch
    import torch.distributed as dist
    from hj3d import dist as hdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "exp4_R16_a3_A4_b2_B2.json")))
        log2R, a, A, b, B = g["generator_args"][1:6]
        Sa, Ta = O.gen_exp4(log2R, a, A, b, B)
        nb, cardR = g["nb"], 1 << log2R
        keys = [np.arange(cardR, dtype=np.uint32), Sa, Ta]
        send, cnts = [], []
        for k in range(3):
            n = len(keys[k])
            lo, hi = rank * n // WORLD, (rank + 1) * n // WORLD
            pairs, counts = partition(keys[k][lo:hi], np.arange(lo, hi, dtype=np.uint32), nb, WORLD)
            send.append(pairs)
            cnts.append(counts)
        sc, rc = hdist.exchange_counts(torch.from_numpy(np.stack(cnts)))
        recv = []
        for k in range(3):
            rbuf = torch.empty((max(sum(rc[k]), 1), 2), dtype=torch.int32)
            got, work = hdist.exchange_pairs_async(torch.from_numpy(send[k].view(np.int32)), sc[k], rc[k], rbuf)
            assert work is None or work.wait()
            recv.append(got.numpy().view(np.uint32))
        out = {}
        for plan in ("Ndu", "Chj"):
            e = O.exp4_plan(recv[0], recv[1], recv[2], nb, plan == "Ndu", keys=(0, 0, 0), rows=(1, 1, 1))
            sums = [e.get(k, 0) for k in EXP4_KEYS] + [e["out"][k] for k in ("sum_a", "sum_b", "sum_c", "sum_h")]
            out[plan] = (hdist.allreduce_sum_u64(sums, "cpu"), hdist.allreduce_xor_u64(e["out"]["xor_h"], "cpu"),
                         [len(r) for r in recv])
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_exp4_co_partitioned_world2():
    """Experiment 4 (Ndu and Chj) split over two ranks by bucket range of the FK hash equals the
    reference binary's fixture exp4_R16_a3_A4_b2_B2: every probe / comparison / unnest counter, c_top
    and the output checksums, after the all-reduce."""
    import json
    import torch.multiprocessing as mp

    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "exp4_R16_a3_A4_b2_B2.json")))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exp4_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for plan in ("Ndu", "Chj"):
        ref = g["plans"][plan]
        tot, x, _ = res[0][plan]
        assert (tot, x) == res[1][plan][:2], plan
        want = [ref["c_probe_RS"], ref["c_probe_RS_cmp"], ref["c_probe_RT"], ref["c_probe_RT_cmp"],
                ref.get("c_unnest_1", 0), ref.get("c_unnest_2", 0), ref["c_top"]]
        assert tot[:7] == want, (plan, tot[:7], want)  # (Chj has no unnest operators: 0, 0)
        assert tot[7:] == [ref["out"][k] for k in ("sum_a", "sum_b", "sum_c", "sum_h")] and x == ref["out"]["xor_h"], plan
        # both ranks own a share of every relation
        assert min(res[0][plan][2] + res[1][plan][2]) > 0
