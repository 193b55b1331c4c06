#!/usr/bin/env python3
"""Diagnostic (not product): which RCCL message shapes carry a config-D-sized chunk intact.

One world-1 RCCL self-exchange through the library (hj3d_comm_exchange) of n random (key, row) pairs,
with the exchange's word type and piece size (bytes, log2) overridden by HJ3D_COMM_WORD /
HJ3D_COMM_PIECE_LOG2 in a diagnostic build (-DHJ3D_COMM_DIAG; read once per process:
scripts/rccl_limits.sh runs one process per setting). argv: pairs [piece_log2 as labelled]. Prints one JSON line:
the setting, the bytes, whether the received buffer equals the sent one, and the first differing
pair index when not."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))


def main():
    import torch
    import hj3d
    n = int(float(sys.argv[1]))
    ctx = hj3d.Context(0)
    comm = hj3d.Comm(ctx, hj3d.Comm.unique_id(ctx), 0, 1)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    send = torch.randint(-2**31, 2**31 - 1, (n, 2), dtype=torch.int32, device="cuda", generator=g)
    recv = torch.full_like(send, -1)
    got, _ = comm.exchange(send, [n], [n], recv, asynchronous=False)
    ctx.sync()
    ok = bool(torch.equal(got, send))
    first = None
    if not ok:
        bad = (got != send).any(dim=1).nonzero()
        first = int(bad[0]) if bad.numel() else None
        nbad = int(bad.numel())
    line = {"pairs": n, "bytes": n * 8, "word": os.environ.get("HJ3D_COMM_WORD", "auto"),
            "piece_log2": int(sys.argv[2]) if len(sys.argv) > 2 else 28,
            "lib": os.path.basename(os.path.dirname(os.environ.get("HJ3D_LIB") or "lib/x")), "intact": ok}
    if not ok:
        line.update({"first_bad_pair": first, "bad_pairs": nbad, "first_bad_byte": first * 8 if first is not None else None})
    print(json.dumps(line), flush=True)
    comm.close()


if __name__ == "__main__":
    main()
