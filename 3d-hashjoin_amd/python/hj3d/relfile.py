"""Binary relation files: generate a relation once, reload it memory-mapped.

The reference generates its relations on every run with one sequential mt19937 stream
(util/GenRandIntVec.cc:72-200, main_experiment1.cc:415-457), which takes minutes at config D's
1e9 tuples. A relation file holds an (n, words) u32 array of structs plus the parameters it was
made from, so a bit-exact reference-generator relation (oracle) or a device-generated one is made
once and then mapped, checked and uploaded in chunks.

Layout: a 4096-byte header (magic ``HJ3DREL1``, then UTF-8 JSON: n, words, key_word, checksum,
meta; zero padded), then n * words little-endian u32 values. The checksum is the
order-dependent u64 sum over rows of mix64(row << 32 | word0) ^ mix64 of the other words (the
same splitmix64 finalizer as include/hj3d.h), computed in chunks.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import numpy as np

MAGIC = b"HJ3DREL1"
HEADER = 4096
CHUNK = 1 << 22  # rows per checksum / upload chunk


def _mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def checksum(rows: np.ndarray, row0: int = 0) -> int:
    """u64 checksum of an (n, words) u32 block whose first row has index row0 (chunkable: the
    checksum of a relation is the sum of its blocks' checksums mod 2^64)."""
    rows = np.asarray(rows, dtype=np.uint32)
    if rows.shape[0] == 0:
        return 0
    idx = np.arange(row0, row0 + rows.shape[0], dtype=np.uint64)
    h = _mix64((idx << np.uint64(32)) | rows[:, 0].astype(np.uint64))
    for w in range(1, rows.shape[1]):
        h ^= _mix64(rows[:, w].astype(np.uint64) + np.uint64(w << 32))
    with np.errstate(over="ignore"):
        return int(h.sum(dtype=np.uint64))


def save(path: str, rows: np.ndarray, key_word: int = 0, meta: Optional[dict] = None) -> dict:
    """Write an (n, words) u32 relation (written in chunks; rows may be a memmap)."""
    rows = np.asarray(rows)
    if rows.ndim != 2 or rows.dtype.itemsize != 4:
        raise ValueError("a relation is an (n, words) array of 4-byte values")
    n, words = rows.shape
    ck = 0
    for a in range(0, n, CHUNK):
        ck = (ck + checksum(rows[a:a + CHUNK].view(np.uint32), a)) & ((1 << 64) - 1)
    head = {"n": int(n), "words": int(words), "key_word": int(key_word), "checksum": ck, "meta": meta or {}}
    blob = MAGIC + json.dumps(head).encode()
    if len(blob) > HEADER:
        raise ValueError("metadata too large for the header")
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(blob + b"\0" * (HEADER - len(blob)))
        for a in range(0, n, CHUNK):
            f.write(np.ascontiguousarray(rows[a:a + CHUNK], dtype=np.uint32).tobytes())
    os.replace(tmp, path)
    return head


def read_header(path: str) -> dict:
    with open(path, "rb") as f:
        blob = f.read(HEADER)
    if not blob.startswith(MAGIC):
        raise ValueError(f"{path}: not an hj3d relation file")
    head = json.loads(blob[len(MAGIC):].rstrip(b"\0").decode())
    if os.path.getsize(path) != HEADER + 4 * head["n"] * head["words"]:
        raise ValueError(f"{path}: truncated relation file")
    return head


def load(path: str, verify: bool = True):
    """(memory-mapped (n, words) u32 array, header). verify: recompute the checksum."""
    head = read_header(path)
    rows = np.memmap(path, dtype=np.uint32, mode="r", offset=HEADER, shape=(head["n"], head["words"]))
    if verify:
        ck = 0
        for a in range(0, head["n"], CHUNK):
            ck = (ck + checksum(rows[a:a + CHUNK], a)) & ((1 << 64) - 1)
        if ck != head["checksum"]:
            raise ValueError(f"{path}: checksum mismatch")
    return rows, head


def to_device(rows: np.ndarray, device="cuda"):
    """Upload a (memory-mapped) relation into one (n, words) int32 device tensor, chunk by chunk
    (host memory stays one chunk)."""
    import torch
    n, words = rows.shape
    out = torch.empty((n, words), dtype=torch.int32, device=device)
    for a in range(0, n, CHUNK):
        out[a:a + CHUNK].copy_(torch.from_numpy(np.array(rows[a:a + CHUNK], dtype=np.uint32).view(np.int32)))
    return out


def cached(path: str, make, key_word: int = 0, meta: Optional[dict] = None):
    """The relation at `path` if it exists and its meta matches, else make() -> rows, saved."""
    if os.path.exists(path):
        try:
            head = read_header(path)
            if head.get("meta") == (meta or {}):
                return load(path)[0]
        except ValueError:
            pass
    rows = make()
    save(path, rows, key_word, meta)
    return load(path, verify=False)[0]
