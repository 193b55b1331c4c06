"""hj3d — Python plumbing over the C ABI of libhj3d.so (include/hj3d.h).

The product is the HIP library; this module only marshals torch device tensors (plain
device pointers and sizes) into the C ABI for tests, the benchmark and the multi-GPU
driver. There is no CPU fallback anywhere: if libhj3d.so is missing or no GPU is
present, every compute entry point raises.

Relations are torch tensors in device memory holding array-of-structs u32 tuples, e.g.
the experiment-1 tuple {k, a, b} (main_experiment1.cc:86) is an (n, 3) int32 tensor.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(os.path.dirname(HERE))  # 3d-hashjoin_amd/
LIB_PATH = os.environ.get("HJ3D_LIB") or os.path.join(PKG_ROOT, "lib", "libhj3d.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "hj3d.h")

HJ3D_OK, HJ3D_EINVAL, HJ3D_ENOMEM, HJ3D_EDEVICE, HJ3D_EUNSUPPORTED, HJ3D_EOVERFLOW = range(6)
HJ3D_ROW_IMPLICIT = 0xFFFFFFFF
HJ3D_CHAIN, HJ3D_NESTED = 0, 1
PROBE_UNIQUE, PROBE_UNNEST, PROBE_EMIT, PROBE_CHECKSUM, PROBE_ACCUMULATE = 0x1, 0x2, 0x4, 0x8, 0x10
T_BUILD, T_PROBE, T_PROBE_KERNEL, T_PARTITION, T_SCATTER, T_HIST = range(6)
OPT_FORCE_DIRECT, OPT_RADIX_MIN, OPT_NESTED_SORT, OPT_SEL_UNFUSED, OPT_PACKED_PROBE = 1, 2, 4, 5, 6
OPT_PROBE_ITEMS = 7
OPT_PK_SLICE, OPT_PK_STAGE, OPT_PK_BUILD, OPT_NESTED_PK, OPT_SYNC_BUILD = 8, 9, 10, 11, 13
OPT_RP_UNFUSED = 15
OPT_DIAG_GBAR = 16
OPT_DIAG_LOOKBACK = 17
SEL_LT, SEL_LE, SEL_GT, SEL_GE, SEL_EQ, SEL_NE, SEL_RANGE = range(7)
SEL_MAX = 4
SEL_OPS = {"<": SEL_LT, "<=": SEL_LE, ">": SEL_GT, ">=": SEL_GE, "==": SEL_EQ, "!=": SEL_NE, "range": SEL_RANGE}

MASK64 = (1 << 64) - 1


class Hj3dError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"hj3d status {status}: {msg}")
        self.status = status


class _Rel(C.Structure):
    _fields_ = [("base", C.c_void_p), ("n", C.c_uint64), ("stride", C.c_uint32), ("key_off", C.c_uint32),
                ("row_off", C.c_uint32), ("reserved", C.c_uint32), ("row_base", C.c_uint64)]


class _Desc(C.Structure):
    _fields_ = [("num_buckets", C.c_uint64), ("bucket_lo", C.c_uint64), ("bucket_hi", C.c_uint64),
                ("kind", C.c_uint32), ("reserved", C.c_uint32)]


class _ProbeRes(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("n_probe", "n_matched", "n_out", "n_cmps", "sum_a", "sum_b", "sum_c",
                                          "sum_h", "xor_h")]


class _Probe2Res(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("c_probe_rs", "c_probe_rs_cmp", "c_probe_rt", "c_probe_rt_cmp",
                                          "c_unnest_1", "c_unnest_2", "c_top", "sum_a", "sum_b", "sum_c", "sum_h",
                                          "xor_h")]


class _SelPred(C.Structure):
    _fields_ = [("word_off", C.c_uint32), ("op", C.c_uint32), ("is_signed", C.c_uint32), ("reserved", C.c_uint32),
                ("lo", C.c_int64), ("hi", C.c_int64)]


class _Stats(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("nb", "empty", "entries", "distinct", "cc0_min", "cc0_max", "cc0_sum",
                                          "cc0_cnt", "cc1_min", "cc1_max", "cc1_sum", "cc1_cnt")]


_lib = None


def lib():
    """Load libhj3d.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libhj3d.so not found at {LIB_PATH}; build it with `make -C 3d-hashjoin_amd` "
                          "or __graft_entry__.build()")
    # torch first: its HIP runtime is then the one libhj3d.so binds to (one runtime per process;
    # with libhj3d.so loaded first, torch and the library ended up on different runtimes and
    # hj3d_ctx_create saw no device)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    p, u64, u32, i32, st = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int, C.c_int
    R, D = C.POINTER(_Rel), C.POINTER(_Desc)
    sig = {
        "hj3d_mix64": (u64, [u64]),
        "hj3d_ctx_create": (st, [i32, p, C.POINTER(p)]),
        "hj3d_ctx_destroy": (None, [p]),
        "hj3d_ctx_set_stream": (st, [p, p]),
        "hj3d_ctx_stream": (p, [p]),
        "hj3d_ctx_sync": (st, [p]),
        "hj3d_last_error": (C.c_char_p, [p]),
        "hj3d_ctx_timing": (st, [p, i32]),
        "hj3d_ctx_set_option": (st, [p, i32, C.c_int64]),
        "hj3d_ctx_timer": (st, [p, i32, C.POINTER(C.c_double), C.POINTER(u64)]),
        "hj3d_ctx_timer_reset": (st, [p]),
        "hj3d_tevent_create": (st, [p, C.POINTER(p)]),
        "hj3d_tevent_record": (st, [p, p]),
        "hj3d_tevent_elapsed": (st, [p, p, C.POINTER(C.c_float)]),
        "hj3d_tevent_destroy": (None, [p]),
        "hj3d_dev_alloc": (st, [p, u64, C.POINTER(p)]),
        "hj3d_dev_free": (st, [p, p]),
        "hj3d_upload": (st, [p, p, p, u64]),
        "hj3d_download": (st, [p, p, p, u64]),
        "hj3d_table_create": (st, [p, D, C.POINTER(p)]),
        "hj3d_table_destroy": (None, [p]),
        "hj3d_table_reserve": (st, [p, p, u64]),
        "hj3d_table_clear": (st, [p, p]),
        "hj3d_build": (st, [p, p, R]),
        "hj3d_build_many": (st, [p, C.POINTER(p), R, u32]),
        "hj3d_table_build_path": (C.c_char_p, [p]),
        "hj3d_table_finish": (st, [p, p]),
        "hj3d_launch_count": (u64, []),
        "hj3d_table_stats": (st, [p, p, C.POINTER(_Stats)]),
        "hj3d_table_size": (st, [p, p, C.POINTER(u64), C.POINTER(u64)]),
        "hj3d_table_export": (st, [p, p, p, p, p, C.POINTER(u64), C.POINTER(u64)]),
        "hj3d_probe": (st, [p, p, R, u32, p, u64]),
        "hj3d_probe_result": (st, [p, C.POINTER(_ProbeRes)]),
        "hj3d_probe2": (st, [p, p, p, R, u32, p, u64]),
        "hj3d_probe2_result": (st, [p, C.POINTER(_Probe2Res)]),
        "hj3d_partition": (st, [p, R, u64, u32, p, p]),
        "hj3d_partition_sel": (st, [p, R, C.POINTER(_SelPred), u32, u64, u32, p, p]),
        "hj3d_partition_strided": (st, [p, R, C.POINTER(_SelPred), u32, u64, u32, p, u64, p]),
        "hj3d_partition_stride": (u64, [u64, u32]),
        "hj3d_part_range": (None, [u64, u32, u32, C.POINTER(u64), C.POINTER(u64)]),
        "hj3d_probe_geometry": (C.c_int, [C.c_void_p, u64, u64, C.POINTER(u32)]),
        "hj3d_comm_counts_cap": (st, [p, p, u32, u64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "hj3d_key_bitmap": (st, [p, R, u64, p, p]),
        "hj3d_bitmap_or_popcount": (st, [p, p, u32, u64, p]),
        "hj3d_select": (st, [p, R, C.POINTER(_SelPred), u32, p, p]),
        "hj3d_probe_sel": (st, [p, p, R, C.POINTER(_SelPred), u32, u32, p, u64]),
        "hj3d_gen_keys": (st, [p, p, u64, u32, u32, u64, u64, u64]),
        "hj3d_gen_fk": (st, [p, p, u64, u32, u32, u64, u32, u64]),
        "hj3d_gen_zipf": (st, [p, p, u64, u32, u32, u64, u32, C.c_double, u64]),
        "hj3d_expected_fk_join": (st, [p, R, R, u64, i32, p]),
        "hj3d_expected_fk_join_gen": (st, [p, R, u64, u64, i32, p]),
        "hj3d_gen_exp1_ref": (st, [u64, u64, i32, C.c_double, u32, p, p, i32]),
        "hj3d_gen_exp4_ref": (st, [u32, u32, u32, u32, u32, p, p, C.POINTER(u64)]),
        "hj3d_runtime_info": (st, [C.c_char_p, u64]),
        "hj3d_stream_copy": (st, [p, p, p, u64, u32, C.POINTER(C.c_double)]),
        "hj3d_comm_unique_id": (st, [p, C.c_char_p]),
        "hj3d_comm_init": (st, [p, C.c_char_p, i32, i32]),
        "hj3d_comm_destroy": (st, [p]),
        "hj3d_comm_rank": (st, [p, C.POINTER(i32), C.POINTER(i32)]),
        "hj3d_comm_counts": (st, [p, p, u32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "hj3d_comm_exchange": (st, [p, p, C.POINTER(C.c_int64), p, C.POINTER(C.c_int64), u64, u32,
                                    C.POINTER(u32)]),
        "hj3d_comm_exchange_strided": (st, [p, p, u64, C.POINTER(C.c_int64), p, C.POINTER(C.c_int64), u64, u32,
                                            C.POINTER(u32)]),
        "hj3d_comm_wait": (st, [p, u32]),
        "hj3d_comm_allreduce_u64": (st, [p, p, u64, i32]),
        "hj3d_comm_allgather": (st, [p, p, p, u64]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def declared_symbols() -> list[str]:
    """Function names declared in include/hj3d.h (the ABI contract)."""
    import re
    text = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(hj3d_[a-z0-9_]+)\s*\(", text)))


def mix64(z: int) -> int:
    z &= MASK64
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & MASK64
    return z ^ (z >> 31)


def pair_hash(a: int, b: int) -> int:
    return mix64(((a & 0xFFFFFFFF) << 32) | (b & 0xFFFFFFFF))


def _torch():
    import torch
    return torch


class Rel:
    """A device relation: AoS u32 tuples in a torch tensor (no copy)."""

    def __init__(self, tensor, key_word: int, row_word: Optional[int] = None, row_base: int = 0, n: Optional[int] = None):
        torch = _torch()
        if not tensor.is_cuda:
            raise ValueError("relations must live in device memory")
        if tensor.dtype not in (torch.int32, torch.uint32) or tensor.dim() != 2 or not tensor.is_contiguous():
            raise ValueError("relation tensor must be a contiguous (n, words) int32 tensor")
        self.tensor = tensor
        words = tensor.shape[1]
        self.c = _Rel(tensor.data_ptr() if tensor.numel() else None, tensor.shape[0] if n is None else n,
                      4 * words, 4 * key_word,
                      HJ3D_ROW_IMPLICIT if row_word is None else 4 * row_word, 0, row_base)

    @property
    def n(self) -> int:
        return self.c.n


@dataclass
class ProbeResult:
    n_probe: int
    n_matched: int
    n_out: int
    n_cmps: int
    sum_a: int
    sum_b: int
    sum_c: int
    sum_h: int
    xor_h: int
    overflow: bool = False


class TimingEvent:
    """A timing event on a context's stream (hj3d_tevent_*: a HIP event without the system-scope
    fence, so recording it does not stall the kernels around it). Same use as
    torch.cuda.Event(enable_timing=True): record(), then a.elapsed_time(b) in ms."""

    def __init__(self, ctx: "Context"):
        self.ctx = ctx
        h = C.c_void_p()
        ctx._check(lib().hj3d_tevent_create(ctx.h, C.byref(h)), "hj3d_tevent_create")
        self.h = h

    def record(self):
        self.ctx._check(lib().hj3d_tevent_record(self.ctx.h, self.h), "hj3d_tevent_record")

    def elapsed_time(self, other: "TimingEvent") -> float:
        ms = C.c_float()
        st = lib().hj3d_tevent_elapsed(self.h, other.h, C.byref(ms))
        if st != 0:
            raise Hj3dError(st, "hj3d_tevent_elapsed")
        return float(ms.value)

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and _lib is not None:
            _lib.hj3d_tevent_destroy(h)
            self.h = None


class Context:
    """hj3d_ctx: a device, the stream every call is enqueued on, scratch, event timers."""

    def __init__(self, device: int = 0, stream=None):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError("hj3d needs a GPU (torch.cuda.is_available() is False)")
        L = lib()
        torch.cuda.set_device(device)
        if stream is None:
            stream = torch.cuda.current_stream(device)
        self.stream = stream
        h = C.c_void_p()
        self._check(L.hj3d_ctx_create(device, C.c_void_p(stream.cuda_stream), C.byref(h)), "hj3d_ctx_create", None)
        self.h = h
        self.device = device

    def _check(self, status: int, what: str, h=-1):
        if status != HJ3D_OK:
            msg = lib().hj3d_last_error(self.h if h == -1 else h)
            raise Hj3dError(status, f"{what}: {msg.decode() if msg else ''}")

    def close(self):
        if getattr(self, "h", None):
            lib().hj3d_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        self._check(lib().hj3d_ctx_sync(self.h), "sync")

    def set_option(self, option: int, value: int):
        self._check(lib().hj3d_ctx_set_option(self.h, option, value), "set_option")

    def force_direct(self, on: bool = True):
        """A/B switch: chaining build/probe without the radix-partitioned kernels."""
        self.set_option(OPT_FORCE_DIRECT, int(on))

    def nested_sort(self, on: bool = True):
        """Nested builds by the LSD key sort instead of the partition + LDS aggregation build."""
        self.set_option(OPT_NESTED_SORT, int(on))

    def radix_min(self, n: int):
        """Smallest probe side (tuples) that takes the radix-partitioned chaining kernels."""
        self.set_option(OPT_RADIX_MIN, int(n))

    def timing(self, mode: int = 1):
        """0 / False: off; 1 / True: every timer; 2: only the kernel spans carried by a dispatch
        (no marker packets between kernels; see hj3d_ctx_timing)."""
        self._check(lib().hj3d_ctx_timing(self.h, int(mode)), "timing")

    def timer(self, phase: int):
        ms, cnt = C.c_double(), C.c_uint64()
        self._check(lib().hj3d_ctx_timer(self.h, phase, C.byref(ms), C.byref(cnt)), "timer")
        return ms.value, cnt.value

    def timer_reset(self):
        self._check(lib().hj3d_ctx_timer_reset(self.h), "timer_reset")

    def build_many(self, tables, rels):
        """Build tables[k] from rels[k] (hj3d_build_many): two nested tables of one geometry take
        one launch sequence (experiment 4's S and T)."""
        n = len(tables)
        th = (C.c_void_p * n)(*[t.h for t in tables])
        rs = (_Rel * n)(*[r.c for r in rels])
        self._check(lib().hj3d_build_many(self.h, th, rs, n), "hj3d_build_many")

    # ---- probes ----
    def probe(self, table: "Table", rel: Rel, unique: bool = False, unnest: bool = False, out=None,
              fetch: bool = True, checksum: bool = True, accumulate: bool = False) -> Optional[ProbeResult]:
        """One probe strand. checksum=False skips the order-independent output checksums (a
        verification aid the reference does not compute); all counters stay exact.
        accumulate=True adds to the previous probe's result (one strand issued in chunks)."""
        flags = (PROBE_UNIQUE if unique else 0) | (PROBE_UNNEST if unnest else 0) | \
                (PROBE_CHECKSUM if checksum else 0) | (PROBE_ACCUMULATE if accumulate else 0)
        ptr, cap = None, 0
        if out is not None:
            flags |= PROBE_EMIT
            ptr, cap = out.data_ptr(), out.numel() * out.element_size() // 8
        self._check(lib().hj3d_probe(self.h, table.h, C.byref(rel.c), flags, ptr, cap), "hj3d_probe")
        return self.probe_result() if fetch else None

    def probe_result(self) -> ProbeResult:
        r = _ProbeRes()
        st = lib().hj3d_probe_result(self.h, C.byref(r))
        if st not in (HJ3D_OK, HJ3D_EOVERFLOW):
            self._check(st, "hj3d_probe_result")
        return ProbeResult(*(getattr(r, f) for f, _ in _ProbeRes._fields_), overflow=st == HJ3D_EOVERFLOW)

    def probe2(self, ts: "Table", tt: "Table", rel: Rel, fetch: bool = True, checksum: bool = True) -> Optional[dict]:
        """The experiment-4 strand. checksum=False leaves out the triple hashes (sum_h, xor_h: a
        verification aid the reference does not compute); counters and row sums stay exact."""
        flags = PROBE_CHECKSUM if checksum else 0
        self._check(lib().hj3d_probe2(self.h, ts.h, tt.h, C.byref(rel.c), flags, None, 0), "hj3d_probe2")
        return self.probe2_result() if fetch else None

    def probe2_result(self) -> dict:
        r = _Probe2Res()
        self._check(lib().hj3d_probe2_result(self.h, C.byref(r)), "hj3d_probe2_result")
        return {f: getattr(r, f) for f, _ in _Probe2Res._fields_}

    # ---- selection pushdown (AlgSelection / AlgDynSelection, algebra.hh:278-358) ----
    def select(self, rel: Rel, preds, out_pairs=None, count=None, fetch: bool = True):
        """Tuples of `rel` whose conjunction of predicates holds, as a stable (key, row) pair
        relation. preds: [(word, op, lo[, hi][, signed])], op in SEL_OPS ("<", "<=", ">", ">=",
        "==", "!=", "range": lo <= v < hi); compared as int32 (the reference's attrval_t) unless
        signed=False. Returns (pairs tensor (n, 2) int32, Rel over it keyed on word 0 with row
        word 1, count); with fetch=False the count stays on the device (count tensor) and the
        Rel covers the capacity (rel.n) until the caller trims it."""
        torch = _torch()
        if len(preds) > SEL_MAX:
            raise ValueError(f"at most {SEL_MAX} predicates")
        arr = _sel_preds(preds)
        dev = f"cuda:{self.device}"
        if out_pairs is None:
            out_pairs = torch.empty((max(rel.n, 1), 2), dtype=torch.int32, device=dev)
        if count is None:
            count = torch.zeros(1, dtype=torch.int64, device=dev)
        self._check(lib().hj3d_select(self.h, C.byref(rel.c), arr, len(preds), out_pairs.data_ptr(),
                                      count.data_ptr()), "hj3d_select")
        if not fetch:
            return out_pairs, Rel(out_pairs, 0, 1, n=rel.n), count
        self.sync()
        n = int(count.item())
        return out_pairs, Rel(out_pairs, 0, 1, n=n), n

    def probe_sel(self, table: "Table", rel: Rel, preds, unique: bool = False, unnest: bool = False, out=None,
                  fetch: bool = True, checksum: bool = True) -> Optional[ProbeResult]:
        """scan(rel) -> selection(preds) -> probe (hj3d_probe_sel): the selection fused into the
        probe partitioner where it applies. n_probe of the result = the passing tuples."""
        if len(preds) > SEL_MAX:
            raise ValueError(f"at most {SEL_MAX} predicates")
        flags = (PROBE_UNIQUE if unique else 0) | (PROBE_UNNEST if unnest else 0) | (PROBE_CHECKSUM if checksum else 0)
        ptr, cap = None, 0
        if out is not None:
            flags |= PROBE_EMIT
            ptr, cap = out.data_ptr(), out.numel() * out.element_size() // 8
        self._check(lib().hj3d_probe_sel(self.h, table.h, C.byref(rel.c), _sel_preds(preds), len(preds), flags, ptr,
                                         cap), "hj3d_probe_sel")
        return self.probe_result() if fetch else None

    def packed_probe(self, on: bool = True):
        """A/B switch: the unique chaining probe on packed pairs (default) or on (hash, row) pairs."""
        self.set_option(OPT_PACKED_PROBE, int(on))

    def probe_items(self, k: int = 0):
        """A/B switch: pairs per lane and chunk of the packed probe's region walk (0 = automatic, 5..8)."""
        self.set_option(OPT_PROBE_ITEMS, int(k))

    def pk_slice_max(self, w: int = 0):
        """Test hook: upper bound on the packed probe's slice width in buckets (0 = LDS-sized); a
        small bound puts small tables on the two-level (k_pk_part + k_pk_split) path."""
        self.set_option(OPT_PK_SLICE, int(w))

    def pk_stage(self, pairs: int = 0):
        """Test hook: the packed partitioner's carry-flush threshold (0 = its whole LDS stage; 1 =
        write the carried partial segments out after every tile)."""
        self.set_option(OPT_PK_STAGE, int(pairs))

    def pk_plan(self, nb_local: int, n_build: int) -> dict:
        """The packed probe's slice geometry for a table of nb_local buckets and n_build entries
        (hj3d_probe_geometry): {W, P, C, W1, P1}."""
        out = (C.c_uint32 * 5)()
        self._check(lib().hj3d_probe_geometry(self.h, nb_local, n_build, out), "hj3d_probe_geometry")
        return dict(zip(("W", "P", "C", "W1", "P1"), list(out)))

    def pk_build(self, on: bool = True):
        """Test hook: chaining builds take the two-level slice build (pk_build) whenever it applies."""
        self.set_option(OPT_PK_BUILD, int(on))

    def rp_unfused(self, on: bool = True):
        """Small build partitions as two launches (histogram, scatter) instead of the fused
        one-launch partition (HJ3D_OPT_RP_UNFUSED; tests and A/B)."""
        self.set_option(OPT_RP_UNFUSED, int(on))

    def diag_gbar(self, ticks: int = 0):
        """Diagnostic (HJ3D_OPT_DIAG_GBAR): the fused build partition's grid barrier times out after
        `ticks` of the 100 MHz clock and its workgroup 0 never arrives, so the barrier fails (tests
        of the failure path; 0 = off)."""
        self.set_option(OPT_DIAG_GBAR, int(ticks))

    def diag_lookback(self, ticks: int = 0):
        """Diagnostic (HJ3D_OPT_DIAG_LOOKBACK): in the nested build on the packed slices, partition 0
        never publishes its count and the look-back waits at most `ticks` of the 100 MHz clock, so
        the build gives up and the sort build replaces the table (tests of that path; 0 = off)."""
        self.set_option(OPT_DIAG_LOOKBACK, int(ticks))

    def sync_build(self, on: bool = True):
        """Nested builds finished inside hj3d_build (HJ3D_OPT_SYNC_BUILD): the build relation may
        be released when the call returns."""
        self.set_option(OPT_SYNC_BUILD, int(on))

    def nested_pk(self, on: bool = True):
        """Nested aggregation builds always on the packed partitioner's slices (the form tables of
        more than 2048 partitions take; tests)."""
        self.set_option(OPT_NESTED_PK, int(on))

    def sel_unfused(self, on: bool = True):
        """A/B switch: hj3d_probe_sel selects first instead of fusing into the partitioner."""
        self.set_option(OPT_SEL_UNFUSED, int(on))

    # ---- exchange / synthetic data ----
    def partition(self, rel: Rel, num_buckets: int, parts: int, out_pairs, counts, preds=None, stride=None):
        """Bucket-range partition of rel into (key, row) pairs per destination (stable); with
        preds, only the tuples passing the selection are partitioned (hj3d_partition_sel).
        stride: the single-pass form for the probe side, order inside a destination not kept,
        destination p's pairs at rows [p * stride, p * stride + counts[p]) of out_pairs
        (hj3d_partition_strided). counts[p] > stride means destination p spilled (its pairs past
        the stride were not written): re-partition without stride (partition_stride(n, parts) is
        the library's bounded stride; stride = rel's tuple count never spills)."""
        if stride is not None:
            if out_pairs.shape[0] < parts * stride:
                raise ValueError("out_pairs holds fewer than parts * stride pairs")
            self._check(lib().hj3d_partition_strided(self.h, C.byref(rel.c), _sel_preds(preds) if preds else None,
                                                     len(preds) if preds else 0, num_buckets, parts,
                                                     out_pairs.data_ptr(), stride, counts.data_ptr()),
                        "hj3d_partition_strided")
            return
        if preds:
            self._check(lib().hj3d_partition_sel(self.h, C.byref(rel.c), _sel_preds(preds), len(preds), num_buckets,
                                                 parts, out_pairs.data_ptr(), counts.data_ptr()), "hj3d_partition_sel")
            return
        self._check(lib().hj3d_partition(self.h, C.byref(rel.c), num_buckets, parts, out_pairs.data_ptr(),
                                         counts.data_ptr()), "hj3d_partition")

    def key_bitmap(self, rel: Rel, domain: int, bitmap, outside=None):
        """Set bit k of `bitmap` (int32 device tensor of >= ceil(domain/32) words, zeroed) for every
        key k < domain of rel; `outside` (int64[1] device tensor) += keys >= domain."""
        if bitmap.numel() * 32 < domain:
            raise ValueError("bitmap too small for the domain")
        self._check(lib().hj3d_key_bitmap(self.h, C.byref(rel.c), domain, bitmap.data_ptr(),
                                          outside.data_ptr() if outside is not None else None), "hj3d_key_bitmap")

    def bitmap_or_popcount(self, bitmaps, count):
        """count (int64[1] device tensor) += popcount of the OR over the rows of `bitmaps`
        ((rows, words) int32 device tensor)."""
        rows, words = bitmaps.shape
        self._check(lib().hj3d_bitmap_or_popcount(self.h, bitmaps.data_ptr(), rows, words, count.data_ptr()),
                    "hj3d_bitmap_or_popcount")

    def num_distinct(self, rel: Rel, domain: int) -> int:
        """#dv of rel's keys (all < domain) on this GPU; synchronous."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        bm = torch.zeros((1, (domain + 31) // 32), dtype=torch.int32, device=dev)
        cnt = torch.zeros(2, dtype=torch.int64, device=dev)
        self.key_bitmap(rel, domain, bm, cnt[1:])
        self.bitmap_or_popcount(bm, cnt[:1])
        self.sync()
        c, out = cnt.tolist()
        if out:
            raise ValueError(f"{out} keys outside [0, {domain})")
        return c

    def stream_copy_peak(self, dst, src, reps: int = 5) -> dict:
        """The box's streaming-copy rate (hj3d_stream_copy: read + write bytes / launch time, the
        best of six copy variants): SURVEY §8(d)'s same-run copy peak. dst, src: device tensors."""
        nbytes = min(dst.numel() * dst.element_size(), src.numel() * src.element_size()) & ~15
        out = (C.c_double * 3)()
        self._check(lib().hj3d_stream_copy(self.h, C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()),
                                             nbytes, reps, out), "stream_copy")
        v = int(out[2])
        return {"copy_peak_GBs": out[0], "copy_median_GBs": out[1], "bytes_copied": nbytes,
                "variant": f"{v % 100} workgroups/CU of 256 threads, 16-B {'non-temporal ' if v >= 100 else ''}"
                           f"loads+stores, best of {reps} launches"}

    def gen_keys(self, tensor, key_word: int, row_base: int, n_keys: int, seed: int):
        """n_keys == 0: identity (k = global row id); else a seeded permutation of [0, n_keys)."""
        self._check(lib().hj3d_gen_keys(self.h, tensor.data_ptr(), tensor.shape[0], 4 * tensor.shape[1],
                                        4 * key_word, row_base, n_keys, seed), "hj3d_gen_keys")

    def gen_fk(self, tensor, key_word: int, row_base: int, fk_max: int, seed: int):
        self._check(lib().hj3d_gen_fk(self.h, tensor.data_ptr(), tensor.shape[0], 4 * tensor.shape[1],
                                      4 * key_word, row_base, fk_max, seed), "hj3d_gen_fk")

    def gen_zipf(self, tensor, key_word: int, row_base: int, fk_max: int, theta: float, seed: int):
        """key column ~ Zipf(theta) over [0, fk_max), value 0 the most frequent (config C)."""
        self._check(lib().hj3d_gen_zipf(self.h, tensor.data_ptr(), tensor.shape[0], 4 * tensor.shape[1],
                                        4 * key_word, row_base, fk_max, float(theta), seed), "hj3d_gen_zipf")

    def expected_fk_join(self, build: Rel, probe: Rel, n_keys: int, swap: bool = False) -> dict:
        torch = _torch()
        res = torch.zeros(8, dtype=torch.int64, device=f"cuda:{self.device}")
        self._check(lib().hj3d_expected_fk_join(self.h, C.byref(build.c), C.byref(probe.c), n_keys, int(swap),
                                                res.data_ptr()), "hj3d_expected_fk_join")
        self.sync()
        return _res5(res.cpu().tolist())

    def expected_fk_join_gen(self, probe: Rel, n_keys: int, key_seed: int, swap: bool = False, res=None):
        """Expected key/FK aggregates for build keys made by gen_keys(n_keys, key_seed); accumulates
        into the device int64[8] tensor `res` when given (multi-GPU), else returns a dict."""
        torch = _torch()
        r = res if res is not None else torch.zeros(8, dtype=torch.int64, device=f"cuda:{self.device}")
        self._check(lib().hj3d_expected_fk_join_gen(self.h, C.byref(probe.c), n_keys, key_seed, int(swap),
                                                    r.data_ptr()), "hj3d_expected_fk_join_gen")
        if res is not None:
            return None
        self.sync()
        return _res5(r.cpu().tolist())


def _sel_preds(preds):
    arr = (_SelPred * max(1, len(preds)))()
    for k, pr in enumerate(preds):
        word, op, lo = pr[0], pr[1], pr[2]
        hi = pr[3] if len(pr) > 3 and pr[3] is not None else 0
        signed = pr[4] if len(pr) > 4 else True
        arr[k] = _SelPred(4 * word, SEL_OPS.get(op, op), int(bool(signed)), 0, int(lo), int(hi))
    return arr


def _res5(v):
    v = [int(x) & MASK64 for x in v]
    return {"n": v[0], "sum_a": v[1], "sum_b": v[2], "sum_h": v[3], "xor_h": v[4]}


def gen_exp1_ref(nR: int, nS: int, skew: bool = False, theta: float = 1.0, t: int = 0, threads: int = 0):
    """The reference's experiment-1 input columns (hj3d_gen_exp1_ref: Experiment1::init,
    main_experiment1.cc:415-457, bit-exact; host only, no GPU): returns numpy u32 (R.k, S.a)."""
    import numpy as np
    Rk = np.empty(nR, dtype=np.uint32)
    Sa = np.empty(max(nS, 1), dtype=np.uint32)
    st = lib().hj3d_gen_exp1_ref(nR, nS, int(bool(skew)), float(theta), t, Rk.ctypes.data, Sa.ctypes.data, threads)
    if st != HJ3D_OK:
        raise Hj3dError(st, "hj3d_gen_exp1_ref: invalid arguments")
    return Rk, Sa[:nS]


def gen_exp4_ref(log2R: int, alpha: int, mult_a: int, beta: int, mult_b: int):
    """The reference's experiment-4 FK columns (hj3d_gen_exp4_ref: Experiment4::init,
    main_experiment4.cc:517-575, bit-exact; host only): returns numpy u32 (S.a, T.a)."""
    import numpy as np
    card = C.c_uint64()
    L = lib()
    st = L.hj3d_gen_exp4_ref(log2R, alpha, mult_a, beta, mult_b, None, None, C.byref(card))
    if st != HJ3D_OK:
        raise Hj3dError(st, "hj3d_gen_exp4_ref: invalid arguments")
    Sa = np.empty(max(card.value, 1), dtype=np.uint32)
    Ta = np.empty(max(card.value, 1), dtype=np.uint32)
    st = L.hj3d_gen_exp4_ref(log2R, alpha, mult_a, beta, mult_b, Sa.ctypes.data, Ta.ctypes.data, C.byref(card))
    if st != HJ3D_OK:
        raise Hj3dError(st, "hj3d_gen_exp4_ref: invalid arguments")
    return Sa[:card.value], Ta[:card.value]


def partition_stride(n: int, parts: int) -> int:
    """Bounded per-destination area of the single-pass exchange partitioner (hj3d_partition_stride):
    mean + 8 sigma of the binomial destination count + 2 tiles, at most n."""
    return int(lib().hj3d_partition_stride(n, parts))


def part_range(num_buckets: int, parts: int, part: int):
    lo, hi = C.c_uint64(), C.c_uint64()
    lib().hj3d_part_range(num_buckets, parts, part, C.byref(lo), C.byref(hi))
    return lo.value, hi.value


def runtime_info() -> str:
    """The HIP runtime (and RCCL) libhj3d.so runs on (hj3d_runtime_info)."""
    buf = C.create_string_buffer(4096)
    lib().hj3d_runtime_info(buf, len(buf))
    return buf.value.decode()


RED_SUM, RED_MAX, RED_MIN = 0, 1, 2
COMM_ID_BYTES = 128


class Comm:
    """libhj3d's RCCL communicator on a Context (hj3d_comm_*): the exchange of the bucket-range
    partitioned join and the merge of per-rank counters, the same entry points
    the C++ hosts call. `uid` is the 128-byte id from Comm.unique_id(ctx) on rank 0, handed to the
    other ranks by any side channel (hj3d.dist.comm_from_torch uses torch.distributed)."""

    def __init__(self, ctx: Context, uid: bytes, rank: int, world: int):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError("communicator id must be 128 bytes")
        self.ctx = ctx
        ctx._check(lib().hj3d_comm_init(ctx.h, uid, rank, world), "hj3d_comm_init")
        self.rank, self.world = rank, world

    @staticmethod
    def unique_id(ctx: Context) -> bytes:
        buf = C.create_string_buffer(COMM_ID_BYTES)
        ctx._check(lib().hj3d_comm_unique_id(ctx.h, buf), "hj3d_comm_unique_id")
        return buf.raw

    def counts(self, counts, recv_cap: Optional[int] = None):
        """All-to-all of per-destination counts, int64 device tensor [C, world] (row c = the counts
        hj3d_partition wrote for chunk c): host lists (send[c][p], recv[c][p]). Synchronous. With
        recv_cap (elements this rank can receive over the chunks), every rank raises together when
        any rank's total exceeds its capacity (hj3d_comm_counts_cap), before any pair exchange."""
        Cn, P = counts.shape
        if P != self.world or not counts.is_contiguous():
            raise ValueError("counts must be a contiguous [chunks, world] int64 tensor")
        snd = (C.c_int64 * (Cn * P))()
        rcv = (C.c_int64 * (Cn * P))()
        cap = MASK64 if recv_cap is None else int(recv_cap)
        self.ctx._check(lib().hj3d_comm_counts_cap(self.ctx.h, counts.data_ptr(), Cn, cap, snd, rcv),
                        "hj3d_comm_counts_cap")
        return ([list(snd[c * P:(c + 1) * P]) for c in range(Cn)], [list(rcv[c * P:(c + 1) * P]) for c in range(Cn)])

    def exchange(self, send, sc, rc, recv_buf, asynchronous: bool = True, send_stride: Optional[int] = None):
        """Grouped send / recv of one chunk of (key, row) pairs (rows of `send` grouped by
        destination, sc[p] rows for peer p; with send_stride, peer p's rows start at p * send_stride)
        into recv_buf (rc[p] rows from peer p, in rank order).
        Returns (received view, ticket or None); wait(ticket) orders the context stream after it."""
        P = self.world
        total = int(sum(rc))
        elem = send.element_size() * (send.shape[1] if send.dim() > 1 else 1)
        if recv_buf.element_size() * (recv_buf.shape[1] if recv_buf.dim() > 1 else 1) != elem:
            raise ValueError("send and receive rows differ in size")
        sca, rca = (C.c_int64 * P)(*sc), (C.c_int64 * P)(*rc)
        t = C.c_uint32()
        self.ctx._check(lib().hj3d_comm_exchange_strided(self.ctx.h, send.data_ptr() if send.numel() else None,
                                                         send_stride or 0, sca,
                                                         recv_buf.data_ptr() if recv_buf.numel() else None, rca,
                                                         recv_buf.shape[0], elem, C.byref(t) if asynchronous else None),
                        "hj3d_comm_exchange_strided")
        return recv_buf[:total], (t.value if asynchronous else None)

    def wait(self, ticket: int):
        self.ctx._check(lib().hj3d_comm_wait(self.ctx.h, ticket), "hj3d_comm_wait")

    def allreduce_u64(self, values, op: int = RED_SUM):
        """u64 counters reduced over ranks (mod 2^64 for the sum). Synchronous."""
        torch = _torch()
        t = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in (int(x) & MASK64 for x in values)],
                         dtype=torch.int64, device=f"cuda:{self.ctx.device}")
        self.ctx._check(lib().hj3d_comm_allreduce_u64(self.ctx.h, t.data_ptr(), t.numel(), op),
                        "hj3d_comm_allreduce_u64")
        self.ctx.sync()
        return [int(x) & MASK64 for x in t.cpu().tolist()]

    def allgather_u64(self, value: int):
        torch = _torch()
        v = int(value) & MASK64
        dev = f"cuda:{self.ctx.device}"
        src = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v], dtype=torch.int64, device=dev)
        dst = torch.empty(self.world, dtype=torch.int64, device=dev)
        self.ctx._check(lib().hj3d_comm_allgather(self.ctx.h, src.data_ptr(), dst.data_ptr(), 8), "hj3d_comm_allgather")
        self.ctx.sync()
        return [int(x) & MASK64 for x in dst.cpu().tolist()]

    def close(self):
        if self.ctx is not None and getattr(self.ctx, "h", None):
            lib().hj3d_comm_destroy(self.ctx.h)
        self.ctx = None


class Table:
    """hj3d_table: a device-resident chaining (HtChaining1) or nested (HtNested1) hash table."""

    def __init__(self, ctx: Context, kind: int, num_buckets: int, bucket_lo: int = 0, bucket_hi: Optional[int] = None):
        self.ctx = ctx
        desc = _Desc(num_buckets, bucket_lo, num_buckets if bucket_hi is None else bucket_hi, kind, 0)
        h = C.c_void_p()
        ctx._check(lib().hj3d_table_create(ctx.h, C.byref(desc), C.byref(h)), "hj3d_table_create")
        self.h = h
        self.kind = kind
        self.num_buckets = num_buckets

    def reserve(self, n: int):
        self.ctx._check(lib().hj3d_table_reserve(self.ctx.h, self.h, n), "hj3d_table_reserve")

    def build(self, rel: Rel):
        self.ctx._check(lib().hj3d_build(self.ctx.h, self.h, C.byref(rel.c)), "hj3d_build")

    def clear(self):
        self.ctx._check(lib().hj3d_table_clear(self.ctx.h, self.h), "hj3d_table_clear")

    def finish(self):
        """Finish a nested build now (hj3d_table_finish): counts read, sort-build fallback run."""
        self.ctx._check(lib().hj3d_table_finish(self.ctx.h, self.h), "hj3d_table_finish")

    def build_path(self, finish: bool = True) -> str:
        """Which build made the table (hj3d_table_build_path); finish=True resolves a pending
        nested build first, else a pending one reads as the started path + "?"."""
        if finish:
            self.finish()
        return lib().hj3d_table_build_path(self.h).decode()

    def stats(self) -> dict:
        s = _Stats()
        self.ctx._check(lib().hj3d_table_stats(self.ctx.h, self.h, C.byref(s)), "hj3d_table_stats")
        return {f: getattr(s, f) for f, _ in _Stats._fields_}

    def close(self):
        if getattr(self, "h", None):
            lib().hj3d_table_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


from .plans import (EXP1_PLANS, exp1_plan, exp1_plan_sharded, exp1_relations_ref, exp4_plan,  # noqa: E402,F401
                    exp4_plan_sharded, exp4_relations_ref, merge_exp4, merge_shard_stats, num_buckets_exp1,
                    num_distinct_sharded)
