"""ctypes front-end for liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker / the timed single-thread CPU
baseline. The product path (``libhj3d.so`` and ``hj3d``) never imports it.

The C restatement it wraps (hj3d_oracle.c) follows the reference entities
listed in that file's header (ht_chaining.hh, ht_nested.hh, algebra.hh,
util/GenRandIntVec.cc, util/zipf_distribution.hh, main_experiment1/4.cc) and is
pinned by tests/golden/ fixtures produced by the real reference.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class _Rel(C.Structure):
    _fields_ = [("base", C.c_void_p), ("n", C.c_uint64), ("stride", C.c_uint32), ("key", C.c_uint32),
                ("row", C.c_uint32), ("pad", C.c_uint32)]


ROW_IMPLICIT = 0xFFFFFFFF


class _Stats(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in (
        "nb", "empty", "entries", "distinct",
        "cc0_min", "cc0_max", "cc0_sum", "cc0_cnt",
        "cc1_min", "cc1_max", "cc1_sum", "cc1_cnt")]


class _Agg(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("n", "sum_a", "sum_b", "sum_c", "sum_h", "xor_h")]


class _PlanRes(C.Structure):
    _fields_ = [("c_build", C.c_uint64), ("c_probe", C.c_uint64), ("c_cmp", C.c_uint64),
                ("c_unnest", C.c_uint64), ("c_top", C.c_uint64), ("reps", C.c_uint64),
                ("build_ns", C.c_double), ("probe_ns", C.c_double),
                ("stats", _Stats), ("out", _Agg)]


class _Exp4Res(C.Structure):
    _fields_ = [("c_probe_rs", C.c_uint64), ("c_probe_rs_cmp", C.c_uint64), ("c_probe_rt", C.c_uint64),
                ("c_probe_rt_cmp", C.c_uint64), ("c_unnest_1", C.c_uint64), ("c_unnest_2", C.c_uint64),
                ("c_top", C.c_uint64), ("reps", C.c_uint64),
                ("build_s_ns", C.c_double), ("build_t_ns", C.c_double), ("probe_ns", C.c_double),
                ("out", _Agg)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle oracle` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        u64, u32, p = C.c_uint64, C.c_uint32, C.c_void_p
        L.orc_mix64.restype = u64
        L.orc_mix64.argtypes = [u64]
        L.orc_colsum.restype = u64
        L.orc_colsum.argtypes = [p, u64]
        L.orc_gen_exp1.restype = u32
        L.orc_gen_exp1.argtypes = [u64, u64, C.c_int, C.c_double, u32, p, p]
        L.orc_gen_exp4.restype = u64
        L.orc_gen_exp4.argtypes = [u32, u32, u32, u32, u32, p, p]
        L.orc_num_distinct.restype = u64
        L.orc_num_distinct.argtypes = [p, u64]
        for name in ("orc_chain_plan", "orc_nested_plan"):
            f = getattr(L, name)
            f.restype = C.c_int
            f.argtypes = [C.POINTER(_Rel), C.POINTER(_Rel), u64, C.c_int, C.c_int, C.c_double, u64,
                          C.POINTER(_PlanRes)]
        L.orc_exp4_plan.restype = C.c_int
        L.orc_exp4_plan.argtypes = [C.POINTER(_Rel)] * 3 + [u64, C.c_int, C.c_int, C.c_double, u64,
                                                             C.POINTER(_Exp4Res)]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def mix64(z: int) -> int:
    return lib().orc_mix64(z)


def colsum(v: np.ndarray) -> int:
    v = np.ascontiguousarray(v, dtype=np.uint32)
    return lib().orc_colsum(_ptr(v), v.size)


def gen_exp1(nR: int, nS: int, skew: bool = False, theta: float = 1.0, t: int = 0):
    """Experiment-1 columns (R.k, S.a) and fkMax, bit-exact with main_experiment1.cc:415-457."""
    Rk = np.empty(nR, dtype=np.uint32)
    Sa = np.empty(nS, dtype=np.uint32)
    fk = lib().orc_gen_exp1(nR, nS, int(skew), float(theta), t, _ptr(Rk), _ptr(Sa))
    return Rk, Sa, fk


def gen_exp4(log2R: int, alpha: int, multA: int, beta: int, multB: int):
    """Experiment-4 FK columns (S.a, T.a), bit-exact with main_experiment4.cc:517-575."""
    n = lib().orc_gen_exp4(log2R, alpha, multA, beta, multB, None, None)
    Sa = np.empty(n, dtype=np.uint32)
    Ta = np.empty(n, dtype=np.uint32)
    lib().orc_gen_exp4(log2R, alpha, multA, beta, multB, _ptr(Sa), _ptr(Ta))
    return Sa, Ta


def num_distinct(v: np.ndarray) -> int:
    v = np.ascontiguousarray(v, dtype=np.uint32)
    return lib().orc_num_distinct(_ptr(v), v.size)


def tuples3(k: np.ndarray, a: np.ndarray) -> np.ndarray:
    """AoS {u32 k, a, b} relation (main_experiment1.cc:86) as an (n, 3) uint32 array."""
    t = np.zeros((len(k), 3), dtype=np.uint32)
    t[:, 0] = k
    t[:, 1] = a
    return t


def tuples2(k: np.ndarray, a: np.ndarray) -> np.ndarray:
    """AoS {u32 k, a} relation (main_experiment4.cc:150) as an (n, 2) uint32 array."""
    t = np.zeros((len(k), 2), dtype=np.uint32)
    t[:, 0] = k
    t[:, 1] = a
    return t


def _rel(t: np.ndarray, key: int, row: int | None = None) -> _Rel:
    t = np.ascontiguousarray(t, dtype=np.uint32)
    return _Rel(_ptr(t) if t.size else None, t.shape[0], t.shape[1], key,
                ROW_IMPLICIT if row is None else row, 0)


@dataclass
class PlanResult:
    c_build: int
    c_probe: int
    c_cmp: int
    c_unnest: int
    c_top: int
    reps: int
    build_ns: float
    probe_ns: float
    stats: dict
    out: dict


def _agg(a: _Agg) -> dict:
    return {f: getattr(a, f) for f, _ in _Agg._fields_}


def _plan(fn, build, bkey, probe, pkey, nb, flag, agg, min_ms, min_reps, brow=None, prow=None) -> PlanResult:
    build = np.ascontiguousarray(build, dtype=np.uint32)
    probe = np.ascontiguousarray(probe, dtype=np.uint32)
    rb, rp = _rel(build, bkey, brow), _rel(probe, pkey, prow)
    res = _PlanRes()
    rc = fn(C.byref(rb), C.byref(rp), nb, int(flag), int(agg), float(min_ms), int(min_reps), C.byref(res))
    if rc != 0:
        raise RuntimeError(f"oracle plan failed rc={rc}")
    st = {f: getattr(res.stats, f) for f, _ in _Stats._fields_}
    return PlanResult(res.c_build, res.c_probe, res.c_cmp, res.c_unnest, res.c_top, res.reps,
                      res.build_ns, res.probe_ns, st, _agg(res.out))


def chain_plan(build, bkey, probe, pkey, nb, unique, agg=True, min_ms=0.0, min_reps=1, brow=None,
               prow=None) -> PlanResult:
    """Chaining build on `build` (key word `bkey`), probe with `probe` (ht_chaining.hh + algebra.hh:555-672).
    brow / prow: word of an explicit row id (exchanged (key,row) pairs), else row = index."""
    return _plan(lib().orc_chain_plan, build, bkey, probe, pkey, nb, unique, agg, min_ms, min_reps, brow, prow)


def nested_plan(build, bkey, probe, pkey, nb, unnest, agg=True, min_ms=0.0, min_reps=1, brow=None,
                prow=None) -> PlanResult:
    """Nested (3D) build/probe(/unnest) (ht_nested.hh + algebra.hh:362-552)."""
    return _plan(lib().orc_nested_plan, build, bkey, probe, pkey, nb, unnest, agg, min_ms, min_reps, brow, prow)


def exp4_plan(R, S, T, nb, nested, agg=True, min_ms=0.0, min_reps=1, keys=(0, 1, 1), rows=(None, None, None)) -> dict:
    """Experiment-4 Ndu (nested=True) / Chj (nested=False); R/S/T are (n,2) {k,a} arrays (keys: the key
    word of R, S, T; rows: their explicit row-id words, None = row index; e.g. received (key, row)
    pairs on a rank of the multi-GPU strand: keys (0, 0, 0), rows (1, 1, 1))."""
    R = np.ascontiguousarray(R, dtype=np.uint32)
    S = np.ascontiguousarray(S, dtype=np.uint32)
    T = np.ascontiguousarray(T, dtype=np.uint32)
    rr, rs, rt = _rel(R, keys[0], rows[0]), _rel(S, keys[1], rows[1]), _rel(T, keys[2], rows[2])
    res = _Exp4Res()
    rc = lib().orc_exp4_plan(C.byref(rr), C.byref(rs), C.byref(rt), nb, int(nested), int(agg), float(min_ms),
                             int(min_reps), C.byref(res))
    if rc != 0:
        raise RuntimeError(f"oracle exp4 failed rc={rc}")
    d = {f: getattr(res, f) for f, _ in _Exp4Res._fields_ if f != "out"}
    d["out"] = _agg(res.out)
    return d


_SEL_CMP = {
    "<": lambda v, lo, hi: v < lo, "<=": lambda v, lo, hi: v <= lo, ">": lambda v, lo, hi: v > lo,
    ">=": lambda v, lo, hi: v >= lo, "==": lambda v, lo, hi: v == lo, "!=": lambda v, lo, hi: v != lo,
    "range": lambda v, lo, hi: (v >= lo) & (v < hi),
}


def select(rel: np.ndarray, key: int, preds) -> np.ndarray:
    """AlgSelection::step / AlgDynSelection::step (algebra.hh:295-300, 335-340): a tuple goes to
    the consumer iff the predicate holds, in scan order. The predicate is the conjunction of
    preds = [(word, op, lo[, hi][, signed])] over u32 tuple words (compared as int32, the
    reference's attrval_t, unless signed=False). Returns the forwarded tuples as (key, row) pairs,
    row = index in `rel` (the tuple's identity: the reference forwards the same tuple pointer)."""
    rel = np.ascontiguousarray(rel, dtype=np.uint32)
    ok = np.ones(rel.shape[0], dtype=bool)
    for pr in preds:
        word, op, lo = pr[0], pr[1], pr[2]
        hi = pr[3] if len(pr) > 3 and pr[3] is not None else 0
        signed = pr[4] if len(pr) > 4 else True
        v = rel[:, word].view(np.int32).astype(np.int64) if signed else rel[:, word].astype(np.int64)
        ok &= _SEL_CMP[op](v, lo, hi)
    rows = np.nonzero(ok)[0].astype(np.uint32)
    return np.stack([rel[rows, key], rows], axis=1).astype(np.uint32) if rows.size else np.zeros((0, 2), np.uint32)
