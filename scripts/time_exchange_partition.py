"""Times the multi-GPU exchange partitioner (hj3d_partition) on one GPU at config-B size.
usage: python scripts/time_exchange_partition.py [parts]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))
import torch  # noqa: E402
import hj3d  # noqa: E402

parts = int(sys.argv[1]) if len(sys.argv) > 1 else 8
nS = 100_000_000
ctx = hj3d.Context(0)
S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
ctx.gen_keys(S, 0, 0, 0, 0)
ctx.gen_fk(S, 1, 0, 80_000_000, 7)
send = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
cnt = torch.zeros(parts, dtype=torch.int64, device="cuda")
rel = hj3d.Rel(S, key_word=1)
for _ in range(2):
    ctx.partition(rel, 80_000_000, parts, send, cnt)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(5):
    ctx.partition(rel, 80_000_000, parts, send, cnt)
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / 5
print(f"hj3d_partition {parts} parts, 1e8 tuples: {ms:.3f} ms  ({nS * 20 / ms / 1e6:.0f} GB/s alg)")
print("counts", cnt.tolist())
