"""Times the multi-GPU exchange partitioners on one GPU at config-B size (1e8 S tuples, 12-B
tuples): the stable two-pass hj3d_partition and the single-pass hj3d_partition_strided.
usage: python scripts/time_exchange_partition.py [parts ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))
import torch  # noqa: E402
import hj3d  # noqa: E402

PEAK = 8000.0  # GB/s
nS = 100_000_000
ctx = hj3d.Context(0)
S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
ctx.gen_keys(S, 0, 0, 0, 0)
ctx.gen_fk(S, 1, 0, 80_000_000, 7)
rel = hj3d.Rel(S, key_word=1)
for parts in [int(a) for a in sys.argv[1:]] or [8]:
    send = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    strided = torch.empty((parts * nS, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(parts, dtype=torch.int64, device="cuda")
    for name, fn in (("stable two-pass", lambda: ctx.partition(rel, 80_000_000, parts, send, cnt)),
                     ("single-pass", lambda: ctx.partition(rel, 80_000_000, parts, strided, cnt, stride=nS))):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            fn()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 5
        gbs = nS * 20 / ms / 1e6
        print(f"{name:16s} {parts:3d} parts, 1e8 tuples: {ms:.3f} ms  ({gbs:.0f} GB/s alg = {gbs / PEAK:.2f} of 8 TB/s)"
              f"  counts {cnt.tolist()[:8]}", flush=True)
    del strided
