"""Multi-GPU exchange for the bucket-range partitioned join.

One process per GPU. Every rank partitions its local slice of a relation into (key, global
row) pairs grouped by the owning rank (owner(bucket) = bucket * P / NB; hj3d_partition on the
GPU), exchanges the per-destination counts, then the pairs. Each rank then builds / probes only
its own bucket range, so the reference's per-bucket semantics (chain order, comparison counts,
statistics) are preserved and the counters simply add up.

Two transports behind the same functions:
- GPU ranks: libhj3d's own RCCL communicator (hj3d.Comm, hj3d_comm_* in include/hj3d.h), the
  implementation the C++ hosts call too. comm_from_torch() creates it (torch.distributed only
  carries the 128-byte id from rank 0) and use_comm() routes the functions below through it:
  counts all-to-all, grouped send / recv of the pairs on the engine's exchange stream (tickets
  instead of host waits), u64 counter all-reduce / all-gather.
- Without a communicator: torch.distributed collectives, host-staged under gloo. This is the CPU
  test transport (tests/test_dist_gloo.py) and the several-ranks-on-one-GPU rehearsal
  (bench.py --rehearse), which RCCL cannot run ("Duplicate GPU": one rank per device).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


_comm = None


def use_comm(comm) -> None:
    """Route the exchange and the counter merges of this process through `comm` (hj3d.Comm), or
    back to torch.distributed with None."""
    global _comm
    _comm = comm


def current_comm():
    """The hj3d.Comm set by use_comm, or None."""
    return _comm


def comm_from_torch(ctx, group=None):
    """An hj3d.Comm over the ranks of the initialised torch.distributed group: rank 0 creates the
    RCCL id, torch.distributed broadcasts it (the only thing it carries), every rank joins."""
    import hj3d
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    obj = [hj3d.Comm.unique_id(ctx) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return hj3d.Comm(ctx, obj[0], rank, world)


class _Ticket:
    """work-handle look-alike of an asynchronous hj3d_comm_exchange: wait() orders the engine's
    stream after the exchange (no host synchronisation)."""

    def __init__(self, comm, t):
        self.comm, self.t = comm, t

    def wait(self):
        self.comm.wait(self.t)


def _host_staged(group=None) -> bool:
    """gloo moves host tensors only: device tensors are staged through host memory (the
    single-GPU rehearsal of the multi-GPU path, bench.py --rehearse)."""
    return dist.get_backend(group) == "gloo"


def exchange(send_pairs: torch.Tensor, send_counts: torch.Tensor, recv_buf: torch.Tensor | None = None,
             group=None) -> torch.Tensor:
    """all_to_all of (n, 2) int32 (key, row) pairs grouped by destination.

    send_counts: int64 tensor [P] on the pairs' device (as written by hj3d_partition).
    Returns the received pairs (a view of recv_buf when it is large enough)."""
    if _comm is not None:
        sc, rc = _comm.counts(send_counts.reshape(1, -1).contiguous())
        total = int(sum(rc[0]))
        if recv_buf is None or recv_buf.shape[0] < total:
            recv_buf = torch.empty((max(total, 1), 2), dtype=send_pairs.dtype, device=send_pairs.device)
        out, _ = _comm.exchange(send_pairs, sc[0], rc[0], recv_buf, asynchronous=False)
        return out
    world = dist.get_world_size(group)
    if _host_staged(group) and send_pairs.is_cuda:
        rb = recv_buf.cpu() if recv_buf is not None else None
        got = exchange(send_pairs.cpu(), send_counts.cpu(), rb, group)
        if recv_buf is not None and recv_buf.shape[0] >= got.shape[0]:
            recv_buf[: got.shape[0]].copy_(got)
            return recv_buf[: got.shape[0]]
        return got.to(send_pairs.device)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc = send_counts.tolist()
    rc = recv_counts.tolist()
    total = int(sum(rc))
    if recv_buf is None or recv_buf.shape[0] < total:
        recv_buf = torch.empty((max(total, 1), 2), dtype=send_pairs.dtype, device=send_pairs.device)
    out = recv_buf[:total]
    assert len(sc) == world
    dist.all_to_all_single(out, send_pairs[: int(sum(sc))], output_split_sizes=rc, input_split_sizes=sc, group=group)
    return out


class ExchangeOverflow(RuntimeError):
    """Raised on EVERY rank when any rank's receive capacity is below what arrives at it."""


def exchange_counts(send_counts: torch.Tensor, group=None, recv_cap: int | None = None):
    """All-to-all of the per-destination counts of several partitioned chunks at once (one
    collective, one host synchronisation for a whole probe strand, instead of one per chunk).

    send_counts: int64 [C, P] (row c = hj3d_partition's counts of chunk c). Returns host lists
    (send[c][p], recv[c][p]): recv[c][p] = pairs rank p sends this rank in chunk c.
    recv_cap: this rank's receive capacity over the C chunks; the ranks agree (one max all-reduce)
    whether any rank is short and then all raise ExchangeOverflow before any pair collective."""
    if _comm is not None:
        import hj3d
        try:
            return _comm.counts(send_counts.contiguous(), recv_cap)
        except hj3d.Hj3dError as e:
            if e.status == hj3d.HJ3D_EOVERFLOW:
                raise ExchangeOverflow(str(e)) from e
            raise
    world = dist.get_world_size(group)
    C = send_counts.shape[0]
    src = send_counts.t().contiguous()  # [P, C]: the block for destination p is contiguous
    if _host_staged(group) and src.is_cuda:
        src = src.cpu()
    recv = torch.empty_like(src)
    dist.all_to_all_single(recv, src, group=group)
    sc = send_counts.cpu().tolist()
    rc = recv.view(world, C).t().cpu().tolist()
    if recv_cap is not None:
        total = sum(sum(r) for r in rc)
        flag = torch.tensor([1 if total > recv_cap else 0], dtype=torch.int64,
                            device=send_counts.device if not _host_staged(group) else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if int(flag.item()):
            raise ExchangeOverflow(f"exchange: {total} pairs arrive at this rank, it holds {recv_cap}"
                                   if total > recv_cap else "exchange: another rank's receive buffer is short")
    return sc, rc


def exchange_pairs_async(send_pairs: torch.Tensor, sc: list[int], rc: list[int], recv_buf: torch.Tensor,
                         group=None, send_stride: int | None = None):
    """The pair all-to-all of one chunk whose counts were exchanged (exchange_counts), left in flight:
    returns (received view, work handle or None for the host-staged gloo rehearsal). recv_buf must
    hold sum(rc) pairs: every rank knows its own receive total before any pair collective starts,
    so a short buffer is the caller's sizing error, reported before the collective (never a hang).
    send_stride: peer p's pairs start at row p * send_stride of send_pairs (the single-pass
    partitioner's layout, Context.partition(..., stride=)); None: back to back."""
    total = int(sum(rc))
    if recv_buf.shape[0] < total:
        raise RuntimeError(f"exchange: receive buffer holds {recv_buf.shape[0]} pairs, {total} arrive")
    if _comm is not None:
        out, t = _comm.exchange(send_pairs, sc, rc, recv_buf, asynchronous=True, send_stride=send_stride)
        return out, _Ticket(_comm, t)
    out = recv_buf[:total]
    if send_stride is not None:  # torch's all-to-all takes the blocks back to back
        send_pairs = torch.cat([send_pairs[p * send_stride:p * send_stride + int(c)] for p, c in enumerate(sc)])
    src = send_pairs[: int(sum(sc))]
    if _host_staged(group) and send_pairs.is_cuda:
        got = torch.empty((total, 2), dtype=send_pairs.dtype)
        dist.all_to_all_single(got, src.cpu(), output_split_sizes=rc, input_split_sizes=sc, group=group)
        out.copy_(got)
        return out, None
    work = dist.all_to_all_single(out, src, output_split_sizes=rc, input_split_sizes=sc, group=group, async_op=True)
    return out, work


def allreduce_stats(st: dict, device) -> dict:
    """HtStatistics of a bucket-range sharded table (each rank's table holds a disjoint bucket range):
    counts add, extremes take max / min, so the result is the single-table statistics."""
    add = ("nb", "empty", "entries", "distinct", "cc0_sum", "cc0_cnt", "cc1_sum", "cc1_cnt")
    out = dict(zip(add, allreduce_sum_u64([st[k] for k in add], device)))
    if _comm is not None:
        import hj3d
        mx = _comm.allreduce_u64([st["cc0_max"], st["cc1_max"]], hj3d.RED_MAX)
        cc1_min = st["cc1_min"] if st["cc1_cnt"] else (1 << 64) - 1
        mn = _comm.allreduce_u64([st["cc0_min"], cc1_min], hj3d.RED_MIN)
        out.update(cc0_max=mx[0], cc1_max=mx[1], cc0_min=mn[0], cc1_min=mn[1])
        return out
    for k in ("cc0_max", "cc1_max"):
        out[k] = int(allreduce_max(float(st[k]), device))
    for k in ("cc0_min", "cc1_min"):
        # ranks whose shard has no non-empty bucket report cc1_min = 0 with cc1_cnt = 0: skip them
        v = st[k] if (k == "cc0_min" or st["cc1_cnt"]) else float(1 << 52)
        out[k] = int(-allreduce_max(-float(v), device))
    return out


def num_distinct(bitmap: torch.Tensor, or_popcount, group=None) -> int:
    """Global number of distinct keys (the #dv pre-pass of SURVEY §8e step 1; the reference sizes
    its build-on-S.a tables by #dv(S.a), main_experiment1.cc:453-454).

    bitmap: this rank's key bitmap (int32 words, bit k set for every local key k; the word count
    a multiple of the world size), e.g. from Context.key_bitmap. The bitmap is all-to-all'ed in
    world equal slices, so rank r receives slice r of every rank's bitmap (1/world of the domain,
    not the whole map as an all-gather would); `or_popcount((world, words/world) tensor) -> int`
    ORs the received slices and counts their bits (Context.bitmap_or_popcount on the GPU); the
    per-rank counts are summed. RCCL has no bitwise-OR reduction, hence the exchange."""
    world = dist.get_world_size(group)
    words = bitmap.numel()
    if words % world:
        raise ValueError(f"bitmap words ({words}) must be a multiple of the world size ({world})")
    src = bitmap.reshape(-1)
    if _comm is not None:
        recv = torch.empty_like(src)
        per = [words // world] * world
        _comm.exchange(src, per, per, recv, asynchronous=False)
        c = int(or_popcount(recv.view(world, words // world)))
        return _comm.allreduce_u64([c])[0]
    if _host_staged(group) and src.is_cuda:
        src = src.cpu()
    recv = torch.empty_like(src)
    dist.all_to_all_single(recv, src, group=group)
    c = int(or_popcount(recv.view(world, words // world)))
    t = torch.tensor([c], dtype=torch.int64, device="cpu" if _host_staged(group) else bitmap.device)
    dist.all_reduce(t, group=group)
    return int(t.item())


def num_distinct_rel(ctx, rel, domain: int, group=None) -> int:
    """num_distinct over the keys (< domain) of every rank's slice `rel`, bitmaps built and
    popcounted by the engine (hj3d_key_bitmap / hj3d_bitmap_or_popcount)."""
    world = dist.get_world_size(group)
    words = (domain + 31) // 32
    words = (words + world - 1) // world * world
    dev = rel.tensor.device
    bm = torch.zeros(words, dtype=torch.int32, device=dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    ctx.key_bitmap(rel, domain, bm, cnt[1:])

    def or_popcount(slices):
        c = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.bitmap_or_popcount(slices.to(dev).contiguous(), c)
        return int(c.item())

    n = num_distinct(bm, or_popcount, group)
    outside = allreduce_sum_u64([int(cnt[1].item())], dev)[0]
    if outside:
        raise ValueError(f"{outside} keys outside [0, {domain})")
    return n


def allreduce_sum_u64(values: list[int], device) -> list[int]:
    """Sum u64 counters over ranks (mod 2^64, as the reference's u64 counters would wrap)."""
    if _comm is not None:
        return _comm.allreduce_u64(values)
    device = "cpu" if _host_staged() else device
    t = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in values], dtype=torch.int64, device=device)
    dist.all_reduce(t)
    return [int(x) & ((1 << 64) - 1) for x in t.tolist()]


def allreduce_xor_u64(value: int, device) -> int:
    if _comm is not None:
        x = 0
        for v in _comm.allgather_u64(value):
            x ^= v
        return x
    device = "cpu" if _host_staged() else device
    world = dist.get_world_size()
    t = torch.tensor([value - (1 << 64) if value >= (1 << 63) else value], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    x = 0
    for o in out:
        x ^= int(o.item()) & ((1 << 64) - 1)
    return x


def allreduce_max(value: float, device) -> float:
    device = "cpu" if _host_staged() else device
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def exp4_join(ctx, plan: str, R: torch.Tensor, S: torch.Tensor, T: torch.Tensor, nb: int, row_base=(0, 0, 0),
              group=None, checksum: bool = True) -> dict:
    """Experiment 4 on this rank of the multi-GPU strand: R {k,a}, S {k,a}, T {k,a} are
    this rank's contiguous slices ((n, 2) int32 device tensors; their first global rows in row_base).
    The three relations are co-partitioned by bucket range of the one FK hash (R on R.k, S and T on
    S.a / T.a: owner(bucket) = bucket * world / nb, hj3d_partition, stable, global rows), their
    counts travel in ONE collective and their pairs in one exchange (three asynchronous pair
    all-to-alls); the rank builds its S and T tables over its bucket range (one hj3d_build_many) and
    runs the two-table probe strand on its R pairs (hj3d_probe2: Ndu, main_experiment4.cc:831-941,
    or Chj, :943-1043). The counters are all-reduced (sums; the triple hash's xor by all-gather), so
    every rank returns the single-table result."""
    import hj3d
    from .plans import EXP4_SUM
    # the ranks of the exchange: libhj3d's communicator when one is set (use_comm), else the group's
    rank, world = (_comm.rank, _comm.world) if _comm is not None else (dist.get_rank(group), dist.get_world_size(group))
    kind = hj3d.HJ3D_NESTED if plan == "Ndu" else hj3d.HJ3D_CHAIN
    dev = R.device
    rels = [hj3d.Rel(R, 0, row_base=row_base[0]), hj3d.Rel(S, 1, row_base=row_base[1]),
            hj3d.Rel(T, 1, row_base=row_base[2])]
    send = [torch.empty((max(r.n, 1), 2), dtype=torch.int32, device=dev) for r in rels]
    cnt = torch.zeros((3, world), dtype=torch.int64, device=dev)
    for k in range(3):
        ctx.partition(rels[k], nb, world, send[k], cnt[k])
    sc, rc = exchange_counts(cnt, group)
    recv = [torch.empty((max(int(sum(rc[k])), 1), 2), dtype=torch.int32, device=dev) for k in range(3)]
    got, works = [], []
    for k in range(3):
        v, w = exchange_pairs_async(send[k], sc[k], rc[k], recv[k], group)
        got.append(v)
        works.append(w)
    for w in works:
        if w is not None:
            w.wait()
    lo, hi = hj3d.part_range(nb, world, rank)
    ts, tt = hj3d.Table(ctx, kind, nb, lo, hi), hj3d.Table(ctx, kind, nb, lo, hi)
    own = [hj3d.Rel(got[k], 0, row_word=1, n=int(sum(rc[k]))) for k in range(3)]
    ctx.build_many([ts, tt], [own[1], own[2]])
    r = ctx.probe2(ts, tt, own[0], checksum=checksum)
    ts.close()
    tt.close()
    out = dict(zip(EXP4_SUM, allreduce_sum_u64([r[k] for k in EXP4_SUM], dev)))
    out["xor_h"] = allreduce_xor_u64(r["xor_h"], dev)
    out["per_rank"] = {"probe_tuples": own[0].n, "build_tuples": own[1].n + own[2].n}
    return out
